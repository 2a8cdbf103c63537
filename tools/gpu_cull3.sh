#!/bin/bash
# Back-face occlusion test (BOPX_VSD_CULL=3): parity of the fused path, then a
# same-box interleaved timing A/B of the cull / queue-order switches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${PAR_K:-fused or raster}" > gpurun_out/par.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/par.log; exit 1; }
tail -1 gpurun_out/par.log
COMBOS="${COMBOS:-0:1 3:1}" REPS=${REPS:-2} bash tools/gpu_envab2.sh
