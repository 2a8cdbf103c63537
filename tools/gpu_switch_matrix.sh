#!/bin/bash
# INTEGRATION.md §4 claims identical results under every runtime switch: the
# fused-VSD / raster / shared-render / point-error parity tests under each
# non-default setting, one pytest run per setting (same process count limits).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for env in "BOPX_VSD_CULL=0" "BOPX_VSD_CULL=3" "BOPX_VSD_CULL=1" "BOPX_VSD_QORDER=0" \
           "BOPX_LAUNCH_ORDER=0" "BOPX_VSD_SPLIT=4" "BOPX_VSD_TAIL=300" "BOPX_SYM_PRUNE=0" \
           "BOPX_ADI_SPLIT=1" "BOPX_ADI_QSPLIT=1" "BOPX_SHARED_RENDER_RATIO=0" \
           "BOPX_MESHLET_CURVE=morton"; do
  env $env timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shared.py \
      tests/test_gpu_configs.py -q -x --timeout 240 --timeout-method thread \
      -k "fused or raster or shared or sym or adi or config or cover" > gpurun_out/sw.log 2>&1 \
      || { echo "$env FAILED"; tail -20 gpurun_out/sw.log; exit 1; }
  echo "$env: $(tail -1 gpurun_out/sw.log)"
done
# host-side switches of the callers (round 4): the record-dict error path, the
# Python scorer and the host depth decoder, against the reference scripts' files
for env in "BOPX_ERRORS_ARRAYS=0" "BOPX_SCORE_NATIVE=0" "BOPX_DEPTH_GPU=0"; do
  env $env timeout -k 10 300 python -u -m pytest tests/test_e2e_errors.py tests/test_scores.py \
      tests/test_gt_side.py \
      -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/sw.log 2>&1 \
      || { echo "$env FAILED"; tail -20 gpurun_out/sw.log; exit 1; }
  echo "$env: $(tail -1 gpurun_out/sw.log)"
done
