#!/bin/bash
# Meshlet curve A/B (BOPX_MESHLET_CURVE=morton vs the default Hilbert order):
# parity, bench, k_vsd workload counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/par.log 2>&1 || { tail -30 gpurun_out/par.log; exit 1; }
tail -1 gpurun_out/par.log
for c in morton hilbert; do
  BOPX_MESHLET_CURVE=$c timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/ml_$c.json 2>gpurun_out/ml_$c.err || { tail gpurun_out/ml_$c.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/ml_$c.json'));print('$c', round(d['value']), {k:round(v['ms'],2) for k,v in d['kernels'].items()})"
  BOPX_MESHLET_CURVE=$c BOPX_LIB=$PWD/bop_toolkit_amd/lib/diag/libbopx_diag.so BOPX_VSD_ABLATE=4 timeout -k 10 200 python tools/vsd_stats.py --tuples 1200 | grep -E "entries|setups|passes" || exit 1
done
