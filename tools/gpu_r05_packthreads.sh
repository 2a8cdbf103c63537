#!/bin/bash
# Packing threads of the depth groups (BOPX_PACK_THREADS) on the 100k e2e job,
# same box; prints the cgroup CPU quota first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05pt}
cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"
for v in ${THREADS:-16 12 8}; do
  BOPX_PACK_THREADS=$v timeout -k 10 400 python tools/e2e_bench.py --images 16667 --ab-depth --ab-group 4096/1024 --warm-reps 1 > gpurun_out/e2e_100k_${TAG}_t$v.json 2> gpurun_out/e2e_100k_${TAG}_t$v.err || { tail -20 gpurun_out/e2e_100k_${TAG}_t$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/e2e_100k_${TAG}_t$v.json'))
g=d['depth_decoder_gt_info']; c=d['depth_decoder_first_run']
print('threads=$v gt_info', d['calc_gt_info_s'], g['pack_c_s'], 'cold', d['eval_bop19_s'], d['errors_s'], c['pack_c_s'])
for k,v in d['ab_depth'].items(): print('  warm', v['eval_bop19_s'], v['errors_s'], v['depth_decoder']['pack_c_s'], v['identical_scores'])"
done
