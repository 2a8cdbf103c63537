#!/bin/bash
# PMC of the device PNG decoder (instruction mix and waits per wave).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/png_pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/png_pmc -o run --output-format csv -- python3 tools/png_bench.py --frames 256 --reps 1 > gpurun_out/png_pmc.log 2>&1 || { tail -30 gpurun_out/png_pmc.log; exit 1; }
f=$(find gpurun_out/png_pmc -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
  if "png" not in r["Kernel_Name"]: continue
  k = r["Kernel_Name"].split("(")[0].split("::")[-1]
  agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
for (k, c), v in sorted(agg.items()):
  print(k, c, "%.4g" % v)
PY
