#!/bin/bash
# 100k e2e with per-event host timelines of the warm runs (tools/e2e_bench.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05t}
timeout -k 10 300 python -u -m pytest tests/test_gpu_png.py tests/test_e2e_errors.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_${TAG}.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_${TAG}.log; exit 1; }
tail -1 gpurun_out/gpu_tests_${TAG}.log
timeout -k 10 480 python tools/e2e_bench.py --images 16667 --ab-depth --ab-group ${DEPTH_GROUPS:-4096/1024} --warm-reps ${WARM_REPS:-2} > gpurun_out/e2e_100k_${TAG}.json 2> gpurun_out/e2e_100k_${TAG}.err || { tail -20 gpurun_out/e2e_100k_${TAG}.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/e2e_100k_${TAG}.json'))
print('cold', d['eval_bop19_s'], d['errors_s'], d['tail'])
for k,v in d['ab_depth'].items(): print(k, v['eval_bop19_s'], v['errors_s'], v['depth_decoder'], v['identical_scores'])"
# the same job under a kernel trace (GPU timeline of the decode and error kernels)
if [ -n "$KTRACE" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/e2e_kt_${TAG} -o run --output-format csv -- python3 tools/e2e_bench.py --images 16667 --ab-depth --ab-group ${KTRACE} --root /tmp/bopx_e2e_kt > gpurun_out/e2e_kt_${TAG}.json 2> gpurun_out/e2e_kt_${TAG}.err || { tail -20 gpurun_out/e2e_kt_${TAG}.err; exit 1; }
  ls -la gpurun_out/e2e_kt_${TAG}/* | head
fi
