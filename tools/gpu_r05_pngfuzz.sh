#!/bin/bash
# Randomised GPU-vs-host depth-PNG parity: the suite's size, then BOPX_PNG_FUZZ streams
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05f}
timeout -k 10 300 python -u -m pytest tests/test_gpu_png_fuzz.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/png_fuzz_${TAG}_suite.txt 2>&1 || { tail -30 gpurun_out/png_fuzz_${TAG}_suite.txt; exit 1; }
tail -1 gpurun_out/png_fuzz_${TAG}_suite.txt
BOPX_PNG_FUZZ=${N:-3000} BOPX_PNG_FUZZ_SEED=${SEED:-2025} timeout -k 10 900 python -u -m pytest tests/test_gpu_png_fuzz.py -m gpu -x -v --timeout 880 --timeout-method thread > gpurun_out/png_fuzz_${TAG}_${N:-3000}.txt 2>&1 || { tail -30 gpurun_out/png_fuzz_${TAG}_${N:-3000}.txt; exit 1; }
tail -3 gpurun_out/png_fuzz_${TAG}_${N:-3000}.txt
