#!/bin/bash
# Tile-parallel mode at the bench's batch (12,504 tuples): default (S = 1) vs
# forced S = 2 and 4; the new split parity test; the batch-size sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "tile_parallel or fused_vsd" > gpurun_out/split_tests.log 2>&1 || { tail -30 gpurun_out/split_tests.log; exit 1; }
tail -1 gpurun_out/split_tests.log
for s in 0 2 4 0 2 4; do
  if [ "$s" = 0 ]; then
    timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_s$s.json 2> gpurun_out/bench_s$s.err || { tail -20 gpurun_out/bench_s$s.err; exit 1; }
  else
    BOPX_VSD_SPLIT=$s timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_s$s.json 2> gpurun_out/bench_s$s.err || { tail -20 gpurun_out/bench_s$s.err; exit 1; }
  fi
  python -c "import json;d=json.load(open('gpurun_out/bench_s$s.json'));print('split $s', round(d['value']), {k:round(v['ms'],3) for k,v in d['kernels'].items()})"
done
timeout -k 10 180 python tools/split_sweep.py > gpurun_out/split_sweep_auto2.json 2>> gpurun_out/split_sweep.err && cat gpurun_out/split_sweep_auto2.json
