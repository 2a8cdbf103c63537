#!/bin/bash
# Depth-PNG decoder change on the box: the PNG GPU tests (+ the randomised
# parity at FUZZ streams), then an interleaved decode-time A/B of
# $PREV (default lib/variants/png_base.so) against the product library over
# batch sizes SIZES (tools/png_occupancy.py), and the PMC instruction mix of
# both at 4,096 frames. Every GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-png}
PREV=${PREV:-bop_toolkit_amd/lib/variants/png_base.so}
timeout -k 10 600 env BOPX_PNG_FUZZ=${FUZZ:-96} python -u -m pytest tests/test_gpu_png.py tests/test_gpu_png_fuzz.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_${TAG}.log 2>&1 || { echo "png tests failed"; tail -30 gpurun_out/gpu_tests_${TAG}.log; exit 1; }
tail -2 gpurun_out/gpu_tests_${TAG}.log
: > gpurun_out/png_ab_${TAG}.txt
for r in $(seq ${REPS:-2}); do
  for v in prev new; do
    if [ $v = prev ]; then L=$PWD/$PREV; else L=$PWD/bop_toolkit_amd/lib/libbopx.so; fi
    BOPX_LIB=$L timeout -k 10 240 python tools/png_occupancy.py --sizes ${SIZES:-1024,4096,16384} --reps 1 > gpurun_out/png_ab_${TAG}_${v}_$r.json 2> gpurun_out/png_ab_${TAG}_${v}_$r.err || { tail -20 gpurun_out/png_ab_${TAG}_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/png_ab_${TAG}_${v}_$r.json'));print('$v $r', [(x['frames'], x['decode_us_per_frame']) for x in d['runs']])" | tee -a gpurun_out/png_ab_${TAG}.txt
  done
done
for v in prev new; do
  if [ $v = prev ]; then L=$PWD/$PREV; else L=$PWD/bop_toolkit_amd/lib/libbopx.so; fi
  BOPX_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM --kernel-include-regex "k_png" -d gpurun_out/pngpmc_${TAG}_$v -o run --output-format csv -- python3 tools/png_occupancy.py --sizes 4096 --reps 0 > gpurun_out/pngpmc_${TAG}_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 gpurun_out/pngpmc_${TAG}_$v.log; exit 1; }
done
TAG=$TAG python3 - <<'PY' | tee -a gpurun_out/png_ab_${TAG}.txt
import csv, glob, collections, os
tag=os.environ["TAG"]
for v in ("prev","new"):
  c=collections.defaultdict(float)
  for path in glob.glob("gpurun_out/pngpmc_%s_%s/**/*counter_collection.csv"%(tag,v), recursive=True):
    for r in csv.DictReader(open(path)):
      c[(r["Kernel_Name"].split("(")[0][-16:], r["Counter_Name"])]+=float(r["Counter_Value"])
  for k in sorted(c): print(v, k, "%.4g per frame" % (c[k]/4096))
PY
echo "png session $TAG done"
