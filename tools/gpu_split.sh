#!/bin/bash
# Tile-parallel VSD mode: GPU parity tests, drop-in per-call latency with the
# split on (default) and off (BOPX_VSD_SPLIT=1), the kernel durations of both
# from a rocprofv3 kernel trace, then the batched bench (unaffected: >= 256 tuples).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 240 python tools/percall_bench.py --calls 300 > gpurun_out/percall_split.json 2> gpurun_out/percall_split.err || { tail -30 gpurun_out/percall_split.err; exit 1; }
cat gpurun_out/percall_split.json
BOPX_VSD_SPLIT=1 timeout -k 10 240 python tools/percall_bench.py --calls 300 > gpurun_out/percall_nosplit.json 2> gpurun_out/percall_nosplit.err || { tail -30 gpurun_out/percall_nosplit.err; exit 1; }
cat gpurun_out/percall_nosplit.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_split -o run --output-format csv -- python3 tools/percall_bench.py --calls 300 > gpurun_out/prof_split.log 2>&1 || { tail -30 gpurun_out/prof_split.log; exit 1; }
BOPX_VSD_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nosplit -o run --output-format csv -- python3 tools/percall_bench.py --calls 300 > gpurun_out/prof_nosplit.log 2>&1 || { tail -30 gpurun_out/prof_nosplit.log; exit 1; }
for d in prof_split prof_nosplit; do echo "== $d"; find gpurun_out/$d -name "*kernel_stats.csv" -exec grep -h "k_vsd\|Name" {} \; ; done
timeout -k 10 300 python bench.py > gpurun_out/bench_split.json 2> gpurun_out/bench_split.err || { tail -30 gpurun_out/bench_split.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_split.json'));print(round(d['value']), {k:round(v['ms'],3) for k,v in d['kernels'].items()})"
timeout -k 10 200 python tools/split_sweep.py 1,4,16,32,64,128,192,256,384,512,768,1024,1536 > gpurun_out/split_sweep_auto3.json 2> gpurun_out/split_sweep.err || { tail -20 gpurun_out/split_sweep.err; exit 1; }
cat gpurun_out/split_sweep_auto3.json
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
