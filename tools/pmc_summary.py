"""Summarise rocprofv3 --pmc counter CSVs: per kernel, mean counter value per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(dirs):
  acc = defaultdict(lambda: defaultdict(list))
  for d in dirs:
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
      for row in csv.DictReader(open(path)):
        name = row.get("Kernel_Name", "?")[:60]
        acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
  for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
      # counters are reported per dispatch and per dimension: sum per dispatch
      print("   %-28s %16.4g   (n=%d)" % (c, sum(v) / max(1, len(set(range(len(v))))) * len(v) / max(1, len(v)), len(v)))


if __name__ == "__main__":
  main(sys.argv[1:])
