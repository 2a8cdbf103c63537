#!/bin/bash
# Round 5: depth-decode batch-size sweep, e2e 100k warm A/B of decode group
# sizes, then every other BASELINE config at whole-job size (1 GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/cfg5; export TMPDIR=/tmp
TAG=${TAG:-r05b}
timeout -k 10 300 python tools/png_occupancy.py > gpurun_out/png_occ_${TAG}.json 2> gpurun_out/png_occ_${TAG}.err || { tail -20 gpurun_out/png_occ_${TAG}.err; exit 1; }
cat gpurun_out/png_occ_${TAG}.json
timeout -k 10 480 python tools/e2e_bench.py --images 16667 --ab-depth --ab-group ${DEPTH_GROUPS:-0,4096,5600,8400} > gpurun_out/e2e_100k_${TAG}.json 2> gpurun_out/e2e_100k_${TAG}.err || { tail -20 gpurun_out/e2e_100k_${TAG}.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/e2e_100k_${TAG}.json'))
print('cold', d['eval_bop19_s'], d['errors_s'])
for k,v in d['ab_depth'].items(): print(k, v['eval_bop19_s'], v['errors_s'], v['depth_decoder']['decode_s'], v['identical_scores'])"
for c in ${CONFIGS:-0 1 2 4 5}; do
  timeout -k 10 420 python bench.py --config $c --steps 5 --warmup 1 > gpurun_out/cfg5/config$c.json 2> gpurun_out/cfg5/config$c.err || { tail -20 gpurun_out/cfg5/config$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/cfg5/config$c.json'));print($c, round(d['value']), {k:round(v['ms'],2) for k,v in d['kernels'].items() if v.get('ms')})"
done
