#!/bin/bash
# One box: full GPU parity suite + smoke on the working tree, same-box A/B of
# lib/variants against it, then the end-to-end run at scale (tools/gpu_e2e_scale.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-combo}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { cat gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
if [ -z "$NO_AB" ]; then TAG=$T bash tools/gpu_ab_quick.sh || exit 1; fi
if [ -n "$E2E" ]; then TAG=$T bash tools/gpu_e2e_scale.sh || exit 1; fi
