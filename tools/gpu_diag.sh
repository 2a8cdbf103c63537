#!/bin/bash
# k_vsd workload counters (ABLATE=4) and phase clocks (ABLATE=8) of the diag
# build on the configs[3] bench workload (12,504 tuples unless TUPLES is set).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
LIB=${LIB:-bop_toolkit_amd/lib/diag/libbopx_diag.so}
for ab in 4 8; do
  BOPX_LIB=$PWD/$LIB BOPX_VSD_ABLATE=$ab timeout -k 10 300 python tools/vsd_stats.py --tuples ${TUPLES:-12504} ${EXTRA} > gpurun_out/diag_ab$ab.log 2>&1 || { tail -20 gpurun_out/diag_ab$ab.log; exit 1; }
  grep -E "per tuple|phase|ROI" gpurun_out/diag_ab$ab.log
done
