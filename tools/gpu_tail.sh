#!/bin/bash
# Hybrid tail split of large batches (BOPX_VSD_TAIL): parity with the tail on,
# then the 12,504-tuple bench A/B over tail sizes, interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
BOPX_VSD_TAIL=300 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "tile_parallel or fused_vsd or batch_evaluator" > gpurun_out/tail_tests.log 2>&1 || { tail -30 gpurun_out/tail_tests.log; exit 1; }
tail -1 gpurun_out/tail_tests.log
: > gpurun_out/tail_ab.txt
for rep in 1 2; do
  for t in 0 512 1024 2048; do
    BOPX_VSD_TAIL=$t timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_t$t.json 2> gpurun_out/bench_t$t.err || { tail -20 gpurun_out/bench_t$t.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bench_t$t.json'));print('tail $t', round(d['value']), {k:round(v['ms'],3) for k,v in d['kernels'].items()})" | tee -a gpurun_out/tail_ab.txt
  done
done
