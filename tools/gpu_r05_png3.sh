#!/bin/bash
# k_png_inflate change check: PNG GPU tests, the randomised PNG parity at N
# streams, then an interleaved decode A/B against lib/variants/png_prev.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05q}
timeout -k 10 300 python -u -m pytest tests/test_gpu_png.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_png_${TAG}.log 2>&1 || { echo "png tests failed"; tail -30 gpurun_out/gpu_png_${TAG}.log; exit 1; }
tail -1 gpurun_out/gpu_png_${TAG}.log
BOPX_PNG_FUZZ=${N:-3000} BOPX_PNG_FUZZ_SEED=${SEED:-77} timeout -k 10 600 python -u -m pytest tests/test_gpu_png_fuzz.py -m gpu -x -q --timeout 580 --timeout-method thread > gpurun_out/png_fuzz_${TAG}.txt 2>&1 || { echo "png fuzz failed"; tail -30 gpurun_out/png_fuzz_${TAG}.txt; exit 1; }
tail -1 gpurun_out/png_fuzz_${TAG}.txt
for r in 1 2 3; do
  for v in prev new; do
    if [ $v = prev ]; then L=$PWD/bop_toolkit_amd/lib/variants/png_prev.so; else L=$PWD/bop_toolkit_amd/lib/libbopx.so; fi
    BOPX_LIB=$L timeout -k 10 240 python tools/png_occupancy.py --sizes ${SIZES:-4096,16384} --reps 1 > gpurun_out/png_ab_${TAG}_${v}_$r.json 2> gpurun_out/png_ab_${TAG}_${v}_$r.err || { tail -20 gpurun_out/png_ab_${TAG}_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/png_ab_${TAG}_${v}_$r.json'));print('$v $r', [(x['frames'], x['decode_us_per_frame']) for x in d['runs']])"
  done
done
