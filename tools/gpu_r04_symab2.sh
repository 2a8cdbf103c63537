#!/bin/bash
# Round 4: k_sym_error occupancy variants (MSPD at 6 vs 5 waves, MSSD at 8,
# MSSD staging 1,024): symmetry parity tests on the product, then the A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py -m gpu -q -x --timeout 240 --timeout-method thread -k "sym or config or point" > gpurun_out/symab2_parity.log 2>&1 || { tail -20 gpurun_out/symab2_parity.log; exit 1; }
tail -1 gpurun_out/symab2_parity.log
TAG=symab2 CHECK="mssdw8" CHECK_K="sym" bash tools/gpu_ab_quick.sh
