#!/bin/bash
# Tile-parallel mode in every cost mode: GPU tests, smoke, bench, then the
# end-to-end drop-in pipeline (calc_gt_info + eval_bop19_pose) with the split
# on (default) and off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -30 gpurun_out/bench_final.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_final.json'));print(round(d['value']), {k:round(v['ms'],3) for k,v in d['kernels'].items()})"
timeout -k 10 400 python tools/e2e_bench.py --images 2000 > gpurun_out/e2e_split.json 2> gpurun_out/e2e_split.err || { tail -30 gpurun_out/e2e_split.err; exit 1; }
cat gpurun_out/e2e_split.json
BOPX_VSD_SPLIT=1 timeout -k 10 400 python tools/e2e_bench.py --images 2000 > gpurun_out/e2e_nosplit.json 2> gpurun_out/e2e_nosplit.err || { tail -30 gpurun_out/e2e_nosplit.err; exit 1; }
cat gpurun_out/e2e_nosplit.json
