#!/bin/bash
# Parity tests, then A/B of lib/variants against the product library, then k_vsd counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 600 bash tools/variants.sh || exit 1
BOPX_LIB=$PWD/bop_toolkit_amd/lib/diag/libbopx_diag.so BOPX_VSD_ABLATE=4 timeout -k 10 200 python tools/vsd_stats.py --tuples 1200 || exit 1
