#!/bin/bash
# Native scene_gt / scene_gt_info lists: the GT-side, e2e, scorer and PNG GPU
# tests, then the 100k e2e job with the json path (BOPX_GT_LISTS=0) and the
# native lists, same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05gl}
timeout -k 10 400 python -u -m pytest tests/test_gt_side.py tests/test_e2e_errors.py tests/test_scores.py tests/test_gpu_fuzz.py tests/test_gpu_png.py tests/test_gt_lists.py -m "gpu or not gpu" -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_${TAG}.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_${TAG}.log; exit 1; }
tail -1 gpurun_out/gpu_tests_${TAG}.log
for v in 0 1; do
  BOPX_GT_LISTS=$v timeout -k 10 400 python tools/e2e_bench.py --images 16667 --ab-depth --ab-group 4096/1024 --warm-reps ${WARM_REPS:-2} > gpurun_out/e2e_100k_${TAG}_lists$v.json 2> gpurun_out/e2e_100k_${TAG}_lists$v.err || { tail -20 gpurun_out/e2e_100k_${TAG}_lists$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/e2e_100k_${TAG}_lists$v.json'))
print('lists=$v gt_info', d['calc_gt_info_s'], 'cold', d['eval_bop19_s'], d['errors_s'], d['tail'])
for k,v in d['ab_depth'].items(): print(k, v['eval_bop19_s'], v['errors_s'], v['tail'], v['identical_scores'])"
done
python -c "
import json; a=json.load(open('gpurun_out/e2e_100k_${TAG}_lists0.json')); b=json.load(open('gpurun_out/e2e_100k_${TAG}_lists1.json'))
print('same AR', a['ar']==b['ar'])"
