#!/usr/bin/env python
"""Per-kernel resource usage of a HIP source for gfx950 (VGPRs, AGPRs, SGPRs,
scratch bytes per lane, LDS bytes, occupancy in waves per SIMD), from the
compiler's kernel-resource-usage remarks, with the product Makefile's flags.

    python tools/kernel_resources.py bop_toolkit_amd/csrc/kern_vsd.hip [regex]
    python tools/kernel_resources.py A.hip B.hip [regex]   # side by side
"""
import os
import re
import subprocess
import sys
import tempfile

FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-fast-math", "--cuda-device-only",
         "-Rpass-analysis=kernel-resource-usage"]


def resources(src, extra=()):
  with tempfile.TemporaryDirectory() as d:
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "-c", src, "-o",
                        os.path.join(d, "k.o")], capture_output=True, text=True)
  if r.returncode:
    sys.exit(r.stderr[-3000:])
  out, cur = {}, None
  for line in r.stderr.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|"
                  r"LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
      continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
      cur = out.setdefault(v, {})
    elif cur is not None:
      cur[k.split(" ")[0]] = v
  return out


def main():
  args = [a for a in sys.argv[1:] if a.endswith((".hip", ".cpp"))]
  pat = re.compile(([a for a in sys.argv[1:] if a not in args] or ["."])[0])
  tabs = [resources(a) for a in args]
  cols = ("VGPRs", "AGPRs", "TotalSGPRs", "ScratchSize", "LDS", "Occupancy")
  for name in tabs[0]:
    if not pat.search(name):
      continue
    row = " | ".join(" ".join("%s=%s" % (c[:5], t.get(name, {}).get(c, "-")) for c in cols)
                     for t in tabs)
    print("%-60s %s" % (name[:60], row))


if __name__ == "__main__":
  main()
