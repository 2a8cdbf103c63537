#!/usr/bin/env python
"""Static instruction census of a gfx950 kernel from its assembly.

    python tools/isa_census.py [--kernel MANGLED] [--asm FILE] [--counts diag.json]

Compiles kern_vsd.hip to assembly with line tables (-gline-tables-only does
not change the generated code: the tool checks the instruction stream against
a build without it), splits the kernel into basic blocks, reads LLVM's loop
annotations (header, depth, parent) and the .loc line of every instruction,
and classifies instructions the way the SQ counters do (SQ_INSTS_VALU,
_SALU, _LDS, _VMEM, _SMEM, _BRANCH). Each block is assigned to a phase of
k_vsd by the source line of its instructions (PHASES below) and to its
innermost loop.

With --counts (per-tuple wave-level trip counts of the loops, written by
tools/vsd_stats.py --census from the diag build's counters) the static count
of every loop body is multiplied by the loop's trip count, giving per-phase
dynamic instruction estimates per tuple to set beside the PMC totals.
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "bop_toolkit_amd", "csrc", "kern_vsd.hip")
KERNEL = "_ZN4bopx5k_vsdILi0ELi1ELi10EEEvNS_7VsdArgsE"  # k_vsd<0,1,10>: the bench's instantiation
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-fast-math", "--cuda-device-only", "-S"]

# Source ranges -> phase (file, first line, last line, phase); first match wins.
PHASES = [
    ("raster.h", 357, 406, "walk"),               # r_walk_row_max
    ("kern_vsd.hip", 1049, 1092, "walk"),         # windows, passes, owner lookup, record reads
    ("raster.h", 324, 341, "setup"),              # r_make_row
    ("raster.h", 182, 231, "setup"),              # r_setup_touching
    ("raster.h", 40, 46, "rcp"),                  # rcp_rn (set-up, staging, pixel pass)
    ("raster.h", 254, 305, "slow_raster"),        # r_raster (large / irregular triangles)
    ("kern_vsd.hip", 989, 1048, "setup"),         # chunk loop, row numbering, records
    ("raster.h", 62, 78, "staging"),              # r_vertex
    ("raster.h", 235, 241, "compaction"),         # r_touches
    ("kern_vsd.hip", 971, 988, "compaction"),
    ("kern_vsd.hip", 341, 386, "cull"),           # occlusion-test regions (cull modes)     # bbox test + ballot compaction
    ("kern_vsd.hip", 854, 970, "staging"),        # claim, queue words, loads, transform, cull
    ("kern_vsd.hip", 1093, 1098, "setup"),
    ("kern_vsd.hip", 1099, 1103, "list"),         # list-ahead
    ("kern_vsd.hip", 775, 816, "list"),           # list_tile
    ("kern_vsd.hip", 1104, 1144, "coeffs_touch"),  # touch loads, coefficients, barrier
    ("kern_vsd.hip", 1145, 1178, "pixel_compaction"),
    ("kern_vsd.hip", 86, 106, "pixel"),           # dist_of / visib
    ("kern_vsd.hip", 72, 84, "pixel"),            # sqrt_depth
    ("kern_vsd.hip", 138, 190, "pixel"),          # filter
    ("kern_vsd.hip", 1179, 1316, "pixel"),
    ("kern_vsd.hip", 817, 853, "tile_loop"),
    ("kern_vsd.hip", 1317, 1422, "epilogue"),
    ("kern_vsd.hip", 496, 774, "prologue"),       # rectangles, ROI, thresholds, clears
    ("kern_vsd.hip", 200, 340, "prologue"),       # step_threshold, meshlet_rect, wave max
]


def phase_of(loc):
  if loc is None:
    return "?"
  f, line = loc
  for pf, a, b, name in PHASES:
    if f == pf and a <= line <= b:
      return name
  if f.startswith("amd_") or f.startswith("__clang"):
    return "lib"
  return "other:%s:%d" % (f, line)


def iclass(op):
  if op.startswith("ds_"):
    return "LDS"
  if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
    return "VMEM"
  if op.startswith(("s_load", "s_buffer_load", "s_store", "s_dcache", "s_memtime", "s_memrealtime")):
    return "SMEM"
  if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc", "s_getpc")):
    return "BRANCH"
  if op.startswith(("s_waitcnt", "s_barrier", "s_nop", "s_setprio", "s_endpgm", "s_sleep",
                    "s_sethalt", "s_trap", "s_wait", "s_delay_alu", "s_inst_prefetch")):
    return "OTHER"
  if op.startswith("s_"):
    return "SALU"
  if op.startswith("v_"):
    return "VALU"
  return "OTHER"


def compile_asm(out, line_tables=True):
  cmd = ["/opt/rocm/bin/hipcc"] + FLAGS + (["-gline-tables-only"] if line_tables else []) + [
      "-o", out, SRC]
  subprocess.check_call(cmd, stderr=subprocess.DEVNULL)


def parse(path, kernel):
  """Blocks of `kernel`: dicts with label, loop header (innermost), depth,
  parent headers, and instructions [(op, (file, line))]."""
  files, blocks = {}, []
  on = False
  loc = None
  pending = None  # comment lines of the current block label
  for raw in open(path):
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', raw)
    if m:
      files[int(m.group(1))] = os.path.basename(m.group(3) or m.group(2))
    if raw.startswith(kernel + ":"):
      on = True
      blocks.append({"label": "entry", "comment": "", "insts": []})
      continue
    if not on:
      continue
    if raw.startswith(".Lfunc_end"):
      break
    m = re.match(r'(\.LBB\d+_\d+|; %bb\.\d+):\s*(?:;(.*))?$', raw.rstrip("\n"))
    if m:
      lab = m.group(1)
      lab = lab[2:] if lab.startswith(".L") else "bb." + lab.split(".")[-1]
      blocks.append({"label": lab, "comment": (m.group(2) or "").strip(), "insts": []})
      pending = blocks[-1]
      continue
    if pending is not None and re.match(r"\s+;", raw) and not blocks[-1]["insts"]:
      pending["comment"] += " " + raw.strip(" ;\n")
      continue
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", raw)
    if m:
      loc = (files.get(int(m.group(1)), "?"), int(m.group(2)))
      continue
    s = raw.split(";")[0].strip()
    if not s or s.startswith(".") or s.endswith(":"):
      continue
    blocks[-1]["insts"].append((s.split()[0], loc))
  # loop membership from LLVM's annotations
  for b in blocks:
    c = b["comment"]
    hdr = re.search(r"This (?:Inner )?Loop Header: Depth=(\d+)", c)
    inl = re.search(r"in Loop: Header=(BB\d+_\d+) Depth=(\d+)", c)
    parents = re.findall(r"Parent Loop (BB\d+_\d+) Depth=(\d+)", c)
    b["parents"] = [p for p, _ in parents]
    if hdr:
      b["loop"], b["depth"] = b["label"], int(hdr.group(1))
    elif inl:
      b["loop"], b["depth"] = inl.group(1), int(inl.group(2))
    else:
      b["loop"], b["depth"] = None, 0
  # parents of inner blocks: inherit from the header block
  hdrs = {b["label"]: b for b in blocks if b["loop"] == b["label"]}
  for b in blocks:
    if b["loop"] and b["loop"] != b["label"] and b["loop"] in hdrs:
      b["parents"] = hdrs[b["loop"]]["parents"]
  return blocks


def loop_phase(blocks, header):
  """Majority phase of the instructions of a loop's own blocks."""
  cnt = collections.Counter()
  for b in blocks:
    if b["loop"] == header:
      for op, loc in b["insts"]:
        cnt[phase_of(loc)] += 1
  return cnt.most_common(1)[0][0] if cnt else "?"


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--kernel", default=KERNEL)
  ap.add_argument("--asm", default=None, help="assembly with line tables (default: compile)")
  ap.add_argument("--counts", default=None, help="per-tuple loop trip counts (JSON)")
  ap.add_argument("--json", default=None, help="write the census here")
  a = ap.parse_args()
  path = a.asm
  if path is None:
    path = "/tmp/bopx_isa_census_g.s"
    compile_asm(path, True)
    plain = "/tmp/bopx_isa_census.s"
    compile_asm(plain, False)
    x = [(op) for b in parse(path, a.kernel) for op, _ in b["insts"]]
    y = [(op) for b in parse(plain, a.kernel) for op, _ in b["insts"]]
    if x != y:
      sys.exit("line tables changed the generated code; census not valid")
  blocks = parse(path, a.kernel)
  # static counts per (loop, phase, class)
  per_loop = collections.defaultdict(collections.Counter)
  loops = {}
  for b in blocks:
    key = b["loop"] or "<top>"
    loops.setdefault(key, {"depth": b["depth"], "parents": b["parents"], "blocks": 0})
    loops[key]["blocks"] += 1
    for op, loc in b["insts"]:
      per_loop[key][(phase_of(loc), iclass(op))] += 1
  total = collections.Counter()
  for c in per_loop.values():
    for (ph, cl), n in c.items():
      total[cl] += n
  print("kernel %s: %d blocks, %d instructions (%s)" % (
      a.kernel, len(blocks), sum(total.values()),
      ", ".join("%s %d" % kv for kv in sorted(total.items()))))
  counts = json.load(open(a.counts)) if a.counts else {}
  dyn = collections.defaultdict(collections.Counter)
  rows = []
  for key, info in sorted(loops.items(), key=lambda kv: (kv[1]["depth"], kv[0])):
    c = per_loop[key]
    ph = loop_phase(blocks, key) if key != "<top>" else "prologue/epilogue"
    v = sum(n for (p, cl), n in c.items() if cl == "VALU")
    s = sum(n for (p, cl), n in c.items() if cl == "SALU")
    l = sum(n for (p, cl), n in c.items() if cl == "LDS")
    trip = counts.get(key)
    rows.append({"loop": key, "depth": info["depth"], "parents": info["parents"], "phase": ph,
                 "blocks": info["blocks"], "valu": v, "salu": s, "lds": l, "trip_per_tuple": trip})
    print("%-10s d%d %-18s blocks %3d  VALU %4d SALU %4d LDS %3d  parents %s%s" % (
        key, info["depth"], ph, info["blocks"], v, s, l, ",".join(info["parents"]),
        "" if trip is None else "  trips/tuple %.1f" % trip))
    if trip is not None:
      for (p, cl), n in c.items():
        dyn[p][cl] += n * trip
  if counts:
    print("\ndynamic estimate per tuple (static body x wave-level trips):")
    tot = collections.Counter()
    for p, c in sorted(dyn.items(), key=lambda kv: -kv[1]["VALU"]):
      tot.update(c)
      print("  %-18s VALU %9.0f  SALU %9.0f  LDS %8.0f" % (p, c["VALU"], c["SALU"], c["LDS"]))
    print("  %-18s VALU %9.0f  SALU %9.0f  LDS %8.0f" % ("total", tot["VALU"], tot["SALU"],
                                                        tot["LDS"]))
  if a.json:
    with open(a.json, "w") as f:
      json.dump({"kernel": a.kernel, "static_total": total, "loops": rows,
                 "dynamic_per_tuple": {p: dict(c) for p, c in dyn.items()}}, f, indent=1)


if __name__ == "__main__":
  main()
