#!/bin/bash
# VSD parity (tests/test_gpu_parity.py + the randomised scenes of
# tests/test_gpu_fuzz.py, BOPX_FUZZ_CASES each) of variant libraries before an A/B:
#   bash tools/gpu_variant_parity.sh bop_toolkit_amd/lib/variants/A.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for lib in "$@"; do
  n=$(basename "$lib" .so)
  BOPX_LIB=$PWD/$lib BOPX_FUZZ_CASES=${BOPX_FUZZ_CASES:-60} timeout -k 10 400 python -u -m pytest \
    tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/parity_$n.log 2>&1 || { echo "$n parity failed"; tail -30 gpurun_out/parity_$n.log; exit 1; }
  echo "$n: $(tail -1 gpurun_out/parity_$n.log)"
done
