#!/bin/bash
# k_vsd phase clocks (diag builds): the current diag library and, if present, a
# baseline diag library (lib/diag/libbopx_diag_base.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for lib in bop_toolkit_amd/lib/diag/libbopx_diag.so bop_toolkit_amd/lib/diag/libbopx_diag_base.so; do
  [ -f "$lib" ] || continue
  echo "== $lib"
  BOPX_LIB=$PWD/$lib BOPX_VSD_ABLATE=8 timeout -k 10 200 python tools/vsd_stats.py --tuples 1200 | grep -E "phase|ROI" || exit 1
done
