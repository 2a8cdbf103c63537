#!/bin/bash
# Device depth-PNG decoder: parity tests, the throughput probe, and a rocprof
# kernel-time split of the probe (PROF=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_png.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/png_tests.log 2>&1 || { tail -40 gpurun_out/png_tests.log; exit 1; }
tail -3 gpurun_out/png_tests.log
timeout -k 10 300 python -u tools/png_bench.py --frames ${FRAMES:-512} > gpurun_out/png_bench.json 2> gpurun_out/png_bench.err || { tail -30 gpurun_out/png_bench.err; exit 1; }
cat gpurun_out/png_bench.json
if [ "${PROF:-1}" = 1 ]; then
  rm -rf gpurun_out/png_prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/png_prof -o run --output-format csv -- python3 tools/png_bench.py --frames ${FRAMES:-512} --reps 1 > gpurun_out/png_prof.log 2>&1 || { tail -30 gpurun_out/png_prof.log; exit 1; }
  f=$(find gpurun_out/png_prof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/png_kernel_stats.csv; head -5 gpurun_out/png_kernel_stats.csv
fi
