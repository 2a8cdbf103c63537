#!/bin/bash
# rcp exhaustive check, then parity + bench of libbopx.so and lib/variants/*.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -x tools/rcp_exhaustive ]; then timeout -k 10 120 tools/rcp_exhaustive || { echo "rcp check failed"; exit 1; }; fi
timeout -k 10 900 bash tools/variants.sh || exit 1
