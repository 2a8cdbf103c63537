#!/bin/bash
# Inflate chain rewrite + chunked decoder: PNG / e2e / sharded-caller GPU
# tests, interleaved decode A/B against lib/variants/png_prev.so, PMC of both
# PNG kernels, then the 100k e2e.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05g}
timeout -k 10 600 python -u -m pytest tests/test_gpu_png.py tests/test_e2e_errors.py tests/test_gt_side.py tests/test_dist_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_${TAG}.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_${TAG}.log; exit 1; }
tail -2 gpurun_out/gpu_tests_${TAG}.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { cat gpurun_out/smoke_${TAG}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.log
for r in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then L=$PWD/bop_toolkit_amd/lib/variants/png_prev.so; else L=$PWD/bop_toolkit_amd/lib/libbopx.so; fi
    BOPX_LIB=$L timeout -k 10 240 python tools/png_occupancy.py --sizes ${SIZES:-1024,4096,8192,16384} --reps 1 > gpurun_out/png_ab_${TAG}_${v}_$r.json 2> gpurun_out/png_ab_${TAG}_${v}_$r.err || { tail -20 gpurun_out/png_ab_${TAG}_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/png_ab_${TAG}_${v}_$r.json'));print('$v $r', [(x['frames'], x['decode_us_per_frame']) for x in d['runs']])"
  done
done
for v in prev new; do
  if [ $v = prev ]; then L=$PWD/bop_toolkit_amd/lib/variants/png_prev.so; else L=$PWD/bop_toolkit_amd/lib/libbopx.so; fi
  BOPX_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM --kernel-include-regex "k_png" -d gpurun_out/pngpmc_${TAG}_$v -o run --output-format csv -- python3 tools/png_occupancy.py --sizes 4096 --reps 0 > gpurun_out/pngpmc_${TAG}_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 gpurun_out/pngpmc_${TAG}_$v.log; exit 1; }
done
TAG=$TAG python3 - <<'PY'
import csv, glob, collections, os
tag=os.environ["TAG"]
for v in ("prev","new"):
  c=collections.defaultdict(float)
  for path in glob.glob("gpurun_out/pngpmc_%s_%s/**/*counter_collection.csv"%(tag,v), recursive=True):
    for r in csv.DictReader(open(path)):
      c[(r["Kernel_Name"].split("(")[0][-16:], r["Counter_Name"])]+=float(r["Counter_Value"])
  for k in sorted(c): print(v, k, "%.4g per frame" % (c[k]/4096))
PY
timeout -k 10 480 python tools/e2e_bench.py --images 16667 --ab-depth --ab-group ${DEPTH_GROUPS:-4096,8400} > gpurun_out/e2e_100k_${TAG}.json 2> gpurun_out/e2e_100k_${TAG}.err || { tail -20 gpurun_out/e2e_100k_${TAG}.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/e2e_100k_${TAG}.json'))
print('cold', d['eval_bop19_s'], d['errors_s'], d['host_s'], d['tail'])
for k,v in d['timeline'].items(): print('  ', k, v)
for k,v in d['ab_depth'].items(): print(k, v['eval_bop19_s'], v['errors_s'], v['depth_decoder']['decode_s'], v['tail'], v['identical_scores'])"
