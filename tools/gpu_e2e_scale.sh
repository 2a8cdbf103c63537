#!/bin/bash
# End-to-end BOP19 evaluation at the metric's scale: the
# configs[3]-sized job written as PNG + JSON (16,667 images, 100,002 tuples)
# through calc_gt_info + eval_bop19_pose, with a cProfile of the evaluation.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
df -h /tmp | tail -1
IMAGES=${IMAGES:-16667}
timeout -k 10 1000 python -u tools/e2e_bench.py --images $IMAGES --profile ${E2E_ARGS} > gpurun_out/e2e_${TAG:-scale}.json 2> gpurun_out/e2e_${TAG:-scale}.err || { tail -30 gpurun_out/e2e_${TAG:-scale}.err; exit 1; }
cat gpurun_out/e2e_${TAG:-scale}.json
rm -rf /tmp/bopx_e2e
