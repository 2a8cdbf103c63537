#!/bin/bash
# Round 4, final kernels: the switch matrix (work-moving runtime switches and
# the host switches) and the randomised parity runs at 1,000 VSD scenes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_switch_matrix.sh 2>&1 | tee gpurun_out/switch_matrix.txt || exit 1
BOPX_FUZZ_CASES=1000 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -k vsd -q -x --timeout 500 --timeout-method thread > gpurun_out/fuzz1000.log 2>&1 || { tail -20 gpurun_out/fuzz1000.log; exit 1; }
tail -1 gpurun_out/fuzz1000.log
