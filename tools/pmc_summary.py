"""Summarise rocprofv3 --pmc counter CSVs into profiles/<tag>_pmc.json.

    python tools/pmc_summary.py OUT.json DIR [DIR ...]

If a DIR holds meta.json (bench.py with BOPX_BENCH_META: the libbopx.so sha256
and the workload), it is recorded as `_meta`; bench.py uses a summary's
traffic only when both match the run it reports.

Per kernel: mean value per dispatch of every counter collected (each DIR is one
rocprofv3 pass). HBM traffic per launch follows MI355X_MICROARCH.md §HBM:
FETCH_SIZE and WRITE_SIZE are in KiB (TCC_EA0_RDREQ/_WRREQ based); on gfx950
FETCH_SIZE reports half the bytes of a streaming read. The guide calibrates
16 B/lane; tools/hbm_calib.hip calibrates the 4 B/lane loads k_vsd also uses
(profiles/r01_hbm_calib.csv: 1 GiB streamed -> 524,291 KiB at 4 B/lane and
524,298 KiB at 16 B/lane, i.e. x2 for both). Both the raw sum and the
2x-corrected read side are recorded; the corrected one is
`hbm_bytes_per_launch`.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SHORT = {"k_vsd<0>": "k_vsd", "k_vsd<0,": "k_vsd", "k_sym_error<0>": "k_sym_error<MSSD>",
         "k_sym_error<1>": "k_sym_error<MSPD>"}


def short(name):
  for k, v in SHORT.items():
    if k in name:
      return v
  return name.split("(")[0][-60:]


def main(out, dirs):
  per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
  for d in dirs:
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
      for row in csv.DictReader(open(path)):
        k = short(row.get("Kernel_Name", "?"))
        per[k][row["Counter_Name"]][row.get("Dispatch_Id", "0")] += float(row["Counter_Value"])
  res = {}
  for k, cs in per.items():
    r = {c: sum(v.values()) / len(v) for c, v in cs.items()}
    if "FETCH_SIZE" in r and "WRITE_SIZE" in r:
      r["hbm_bytes_raw_per_launch"] = (r["FETCH_SIZE"] + r["WRITE_SIZE"]) * 1024.0
      r["hbm_bytes_per_launch"] = (2.0 * r["FETCH_SIZE"] + r["WRITE_SIZE"]) * 1024.0
    res[k] = r
  metas = []
  for d in dirs:
    try:
      with open(os.path.join(d, "meta.json")) as f:
        metas.append(json.load(f))
    except (OSError, ValueError):
      pass
  if metas and all(m == metas[0] for m in metas):
    res["_meta"] = metas[0]
  with open(out, "w") as f:
    json.dump(res, f, indent=1, sort_keys=True)
  for k, r in res.items():
    if k == "_meta":
      print("_meta", r)
      continue
    print(k)
    for c, v in sorted(r.items()):
      print("   %-30s %16.6g" % (c, v))


if __name__ == "__main__":
  main(sys.argv[1], sys.argv[2:])
