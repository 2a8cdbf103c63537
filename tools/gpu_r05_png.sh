#!/bin/bash
# Inflate change: GPU PNG parity tests, then a same-box interleaved A/B of
# decode time per frame against the previous revision's library
# (lib/variants/png_prev.so, tools/mkvar_patch.sh with REV=...).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05d}
timeout -k 10 400 python -u -m pytest tests/test_gpu_png.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_png_${TAG}.log 2>&1 || { echo "png tests failed"; tail -30 gpurun_out/gpu_png_${TAG}.log; exit 1; }
tail -2 gpurun_out/gpu_png_${TAG}.log
for r in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then L=$PWD/bop_toolkit_amd/lib/variants/png_prev.so; else L=$PWD/bop_toolkit_amd/lib/libbopx.so; fi
    BOPX_LIB=$L timeout -k 10 240 python tools/png_occupancy.py --sizes ${SIZES:-1024,4096,8192,16384} --reps 1 > gpurun_out/png_ab_${TAG}_${v}_$r.json 2> gpurun_out/png_ab_${TAG}_${v}_$r.err || { tail -20 gpurun_out/png_ab_${TAG}_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/png_ab_${TAG}_${v}_$r.json'));print('$v $r', [(x['frames'], x['decode_us_per_frame']) for x in d['runs']])"
  done
done
if [ -n "$E2E" ]; then
  timeout -k 10 480 python tools/e2e_bench.py --images 16667 --ab-depth --ab-group ${DEPTH_GROUPS:-4096,8400} > gpurun_out/e2e_100k_${TAG}.json 2> gpurun_out/e2e_100k_${TAG}.err || { tail -20 gpurun_out/e2e_100k_${TAG}.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/e2e_100k_${TAG}.json'))
print('cold', d['eval_bop19_s'], d['errors_s'], d['host_s'], d['tail'])
for k,v in d['timeline'].items(): print('  ', k, v)
for k,v in d['ab_depth'].items(): print(k, v['eval_bop19_s'], v['errors_s'], v['depth_decoder']['decode_s'], v['tail'], v['identical_scores'])"
fi
