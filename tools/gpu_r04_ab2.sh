#!/bin/bash
# Round 4: exhaustive ulp accuracy of v_sqrt_f32 / v_rcp_f32 (the filter's
# assumptions), then same-box A/B of lib/variants on configs[3] (25k tuples)
# and on the multi-instance configs[5] (20k tuples, shared renders).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./tools/ulp_exhaustive | tee gpurun_out/ulp_exhaustive.txt || exit 1
TAG=ab2 CHECK="${CHECK}" bash tools/gpu_ab_quick.sh || exit 1
REPS=2 BENCH_ARGS="--config 5 --tuples 20000" bash tools/abrun.sh 2>&1 | tee gpurun_out/ab2_config5.txt
