#!/bin/bash
# GPU tests, smoke, then the drop-in per-call latency.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 240 python tools/percall_bench.py --calls 300 > gpurun_out/percall_final.json 2> gpurun_out/percall_final.err || { tail -30 gpurun_out/percall_final.err; exit 1; }
cat gpurun_out/percall_final.json
