#!/bin/bash
# Round 4: k_sym_error variants (per-wave matrices in SGPRs, MSSD staging size):
# the symmetry parity tests on the working tree's library, then the same-box A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py -m gpu -q -x --timeout 240 --timeout-method thread -k "sym or config or point" > gpurun_out/symab_parity.log 2>&1 || { tail -20 gpurun_out/symab_parity.log; exit 1; }
tail -1 gpurun_out/symab_parity.log
TAG=symab bash tools/gpu_ab_quick.sh || exit 1
timeout -k 10 300 python tools/sym_classes.py --config 3 > gpurun_out/sym_classes_uni.txt 2>&1 && cat gpurun_out/sym_classes_uni.txt
