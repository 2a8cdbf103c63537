#!/bin/bash
# PMC of the PNG decode kernels (k_png_inflate / k_png_unfilter) for the
# product library and lib/variants/png_prev.so: instruction mix per frame.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05f}
for v in prev new; do
  if [ $v = prev ]; then L=$PWD/bop_toolkit_amd/lib/variants/png_prev.so; else L=$PWD/bop_toolkit_amd/lib/libbopx.so; fi
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" "SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVES"; do
    i=$((i+1))
    BOPX_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_png" -d gpurun_out/pngpmc_${TAG}_${v}_$i -o run --output-format csv -- python3 tools/png_occupancy.py --sizes 4096 --reps 0 > gpurun_out/pngpmc_${TAG}_${v}_$i.log 2>&1 || { echo "pass $v $i failed"; tail -5 gpurun_out/pngpmc_${TAG}_${v}_$i.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections, os
tag=os.environ.get("TAG","r05f")
for v in ("prev","new"):
  c=collections.defaultdict(float)
  for path in glob.glob("gpurun_out/pngpmc_%s_%s_*/**/*counter_collection.csv"%(tag,v), recursive=True):
    for r in csv.DictReader(open(path)):
      c[(r["Kernel_Name"].split("(")[0][-14:], r["Counter_Name"])]+=float(r["Counter_Value"])
  for k in sorted(c): print(v, k, "%.4g per frame" % (c[k]/4096))
PY
