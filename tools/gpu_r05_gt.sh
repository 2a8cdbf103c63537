#!/bin/bash
# GT side: its GPU tests, then the 100k e2e with calc_gt_info profiled (cProfile)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05g}
timeout -k 10 300 python -u -m pytest tests/test_gt_side.py tests/test_e2e_errors.py tests/test_scores.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_${TAG}.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_${TAG}.log; exit 1; }
tail -1 gpurun_out/gpu_tests_${TAG}.log
timeout -k 10 480 python tools/e2e_bench.py --images 16667 --profile-gt --ab-depth --ab-group 4096/1024 --warm-reps ${WARM_REPS:-2} > gpurun_out/e2e_100k_${TAG}.json 2> gpurun_out/e2e_100k_${TAG}.err || { tail -20 gpurun_out/e2e_100k_${TAG}.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/e2e_100k_${TAG}.json'))
print('gt_info', d['calc_gt_info_s'], 'cold', d['eval_bop19_s'], d['errors_s'], d['tail'])
for k,v in d['ab_depth'].items(): print(k, v['eval_bop19_s'], v['errors_s'], v['tail'], v['identical_scores'])"
head -60 gpurun_out/gt_profile.txt
