#!/bin/bash
# GPU tests of the host pipeline (e2e byte identity, PNG decode, sharded
# callers), then the 100k e2e with a warm A/B of decode group sizes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05c}
timeout -k 10 600 python -u -m pytest tests/test_e2e_errors.py tests/test_gpu_png.py tests/test_dist_gpu.py tests/test_scores.py tests/test_gt_side.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_${TAG}.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_${TAG}.log; exit 1; }
tail -2 gpurun_out/gpu_tests_${TAG}.log
timeout -k 10 480 python tools/e2e_bench.py --images 16667 --ab-depth --ab-group ${DEPTH_GROUPS:-4096,8400,65536} > gpurun_out/e2e_100k_${TAG}.json 2> gpurun_out/e2e_100k_${TAG}.err || { tail -20 gpurun_out/e2e_100k_${TAG}.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/e2e_100k_${TAG}.json'))
print('cold', d['eval_bop19_s'], d['errors_s'], d['host_s'], d['tail'])
for k,v in d['ab_depth'].items(): print(k, v['eval_bop19_s'], v['errors_s'], v['depth_decoder']['decode_s'], v['tail'], v['identical_scores'])"
