#!/bin/bash
# Round 4: certified float32 filter in the VSD pixel pass. Full GPU parity
# suite, a randomised VSD run, same-box A/B against the previous library
# (lib/variants/head.so) and the diag build's phase clocks / exact-path count
# for both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/filt_gpu_tests.log 2>&1 || { tail -30 gpurun_out/filt_gpu_tests.log; exit 1; }
tail -1 gpurun_out/filt_gpu_tests.log
BOPX_FUZZ_CASES=${FUZZ:-300} timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -k "vsd" -x -q --timeout 300 --timeout-method thread > gpurun_out/filt_fuzz.log 2>&1 || { tail -30 gpurun_out/filt_fuzz.log; exit 1; }
tail -1 gpurun_out/filt_fuzz.log
REPS=${REPS:-3} BENCH_ARGS="--tuples 25000" bash tools/abrun.sh 2>&1 | tee gpurun_out/filt_ab.txt || exit 1
for L in bop_toolkit_amd/lib/diagv/head_diag.so bop_toolkit_amd/lib/diag/libbopx_diag.so; do
  echo "== $L"; LIB=$L TUPLES=12504 bash tools/gpu_diag.sh || exit 1
done 2>&1 | tee gpurun_out/filt_diag.txt
