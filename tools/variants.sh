#!/bin/bash
# A/B the k_vsd tile-size variants (built by `make BUILD=.. OUT=../lib/variants/..`).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for lib in bop_toolkit_amd/lib/libbopx.so bop_toolkit_amd/lib/variants/*.so; do
  [ -f "$lib" ] || continue
  BOPX_LIB=$PWD/$lib timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "${VAR_K:-fused or raster}" > gpurun_out/var.log 2>&1 || { echo "$lib parity FAILED"; tail -20 gpurun_out/var.log; exit 1; }
  BOPX_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/var.json 2>gpurun_out/var.err || { tail gpurun_out/var.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/var.json'));print(sys.argv[1], round(d['value']), {k:round(v['ms'],2) for k,v in d['kernels'].items()})" $lib
done
