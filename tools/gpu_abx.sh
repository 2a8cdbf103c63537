#!/bin/bash
# Quick loop for a k_vsd change: fused-VSD / raster parity of the product
# library, then a same-box interleaved A/B against lib/variants/*.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${PAR_K:-fused or raster}" > gpurun_out/par.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/par.log; exit 1; }
tail -1 gpurun_out/par.log
REPS=${REPS:-3} CULLS=${CULLS:-0} timeout -k 10 900 bash tools/abrun.sh
