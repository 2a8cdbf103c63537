#!/bin/bash
# Timing-only ablation of k_vsd: 0 full, 1 no raster, 2 no pixel pass, 3 neither.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for m in 0 1 2 3; do
  BOPX_VSD_ABLATE=$m timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 ${BENCH_ARGS} > gpurun_out/ablate_$m.json 2> gpurun_out/ablate_$m.err || { tail gpurun_out/ablate_$m.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ablate_$m.json'));print('mode $m', {k:round(v['ms'],2) for k,v in d['kernels'].items()})"
done
