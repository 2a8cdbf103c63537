#!/bin/bash
# GIL switch interval while the depth groups are packed (depth_gpu._gil_switch):
# the PNG / e2e GPU tests, then the 100k e2e job with BOPX_GIL_SWITCH_S=0
# (interpreter default, 5 ms) and the default 0.5 ms, same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05gil}
timeout -k 10 300 python -u -m pytest tests/test_gpu_png.py tests/test_e2e_errors.py tests/test_depth_groups.py -m "gpu or not gpu" -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_${TAG}.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_${TAG}.log; exit 1; }
tail -1 gpurun_out/gpu_tests_${TAG}.log
for v in 0 0.0005; do
  BOPX_GIL_SWITCH_S=$v timeout -k 10 400 python tools/e2e_bench.py --images 16667 --ab-depth --ab-group 4096/1024 --warm-reps ${WARM_REPS:-2} > gpurun_out/e2e_100k_${TAG}_sw$v.json 2> gpurun_out/e2e_100k_${TAG}_sw$v.err || { tail -20 gpurun_out/e2e_100k_${TAG}_sw$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/e2e_100k_${TAG}_sw$v.json'))
print('switch=$v gt_info', d['calc_gt_info_s'], d['depth_decoder_gt_info']['pack_s'], 'cold', d['eval_bop19_s'], d['errors_s'], d['depth_decoder_first_run']['pack_s'], d['ar'])
for k,v in d['ab_depth'].items(): print(k, v['eval_bop19_s'], v['errors_s'], v['depth_decoder']['pack_s'], v['identical_scores'])"
done
