#!/bin/bash
# Cyclic GC paused during the bulk builds (inout.gc_paused: results dicts,
# organize) on the 100k e2e job: BOPX_GC_PAUSE=0 then 1, twice, same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05gc}
timeout -k 10 300 python -u -m pytest tests/test_e2e_errors.py tests/test_scores.py -m "gpu or not gpu" -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_${TAG}.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_${TAG}.log; exit 1; }
tail -1 gpurun_out/gpu_tests_${TAG}.log
for v in 0 1 0 1; do
  k=$((k+1))
  BOPX_GC_PAUSE=$v timeout -k 10 400 python tools/e2e_bench.py --images 16667 --ab-depth --ab-group 4096/1024 --warm-reps 1 > gpurun_out/e2e_100k_${TAG}_gc${v}_$k.json 2> gpurun_out/e2e_100k_${TAG}_gc${v}_$k.err || { tail -20 gpurun_out/e2e_100k_${TAG}_gc${v}_$k.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/e2e_100k_${TAG}_gc${v}_$k.json'))
c=d['depth_decoder_first_run']; tl=d['timeline']
print('gc_pause=$v cold', d['eval_bop19_s'], d['errors_s'], 'pack_c', c['pack_c_s'], 'organize', tl.get('organize',{}).get('busy'), 'load_res', tl.get('load_bop_results',{}).get('busy'), 'gt_info', d['calc_gt_info_s'])
for k,v in d['ab_depth'].items(): print('  warm', v['eval_bop19_s'], v['errors_s'], v['identical_scores'])"
done
