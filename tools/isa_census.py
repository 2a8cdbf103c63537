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

# Phases by source anchors (resolved against the current sources, so the
# table survives edits): functions by name (raster.h / kern_vsd.hip device
# functions), and regions of k_vsd from the first line matching `start` to the
# line before the first later line matching `stop`. First match wins.
FUNCS = {  # device function -> phase
    "rcp_rn": "rcp", "r_vertex": "staging", "r_setup_touching": "setup", "r_touches": "compaction",
    "r_raster": "slow_raster", "r_q": "slow_raster", "r_make_row": "setup",
    "r_walk_row_max": "walk", "vsd_exact_px": "exact", "sqrt_depth": "pixel", "dist_of": "pixel",
    "visib19t": "pixel", "vsd_filter_px": "pixel", "filt_a": "coeffs_touch",
    "filt_b": "coeffs_touch", "filt_thr": "prologue", "step_threshold": "prologue",
    "meshlet_rect": "prologue", "wave_max_nonneg_f32": "prologue", "region_min8": "cull",
    "region_covered": "cull", "make_region": "cull", "wave_incl_scan": "setup",
    "r_regular": "large", "r_floor_div256": "slow_raster",
    "wave_sum_u32": "epilogue", "wave_sum_f64": "epilogue",
}
REGIONS = [  # (start, stop, phase) inside k_vsd
    ("auto raster_tile = [&]", "for (int claimed = 0;; claimed = 1)", "tile_loop"),
    ("for (int t = sp, it = 0;", "if constexpr (COST == kCostRender) return;", "tile_loop"),
    ("auto step_exact = [&]", "auto vsd_px = [&]", "exact"),
    ("if (unc) {  // undo", "} else {  // tlinear", "exact"),
    ("for (int wb = 0; wb <", "VSD_STAMP(11);", "walk"),
    ("for (int c0 = 0; c0 <", "for (int wb = 0; wb <", "setup"),
    ("VSD_STAMP(11);", "}  // rounds (kStream)", "setup"),
    ("int cnt = 0;", "VSD_STAMP(9);", "compaction"),
    ("for (int claimed = 0;; claimed = 1)", "int cnt = 0;", "staging"),
    ("auto list_tile = [&]", "for (int t = sp, it = 0;", "list"),
    ("}  // rounds (kStream)", "// Touch the test-depth lines", "list"),
    ("// Touch the test-depth lines", "// 3. per-pixel distances", "coeffs_touch"),
    ("// 3. per-pixel distances", "// step cost: the certified", "pixel_compaction"),
    ("// step cost: the certified", "// 4. workgroup reduction", "pixel"),
    ("// 4. workgroup reduction", "hipError_t read_vsd_stats", "epilogue"),
    ("void k_vsd(VsdArgs a) {", "// 2a. list the (pose, meshlet)", "prologue"),
]
# Loops: the region (or function) holding the loop's header block -> the diag
# counter of its wave-level trip count (tools/vsd_stats.py "wave" keys, per
# tuple and summed over the 8 waves).
LOOP_REGIONS = [
    ("func", "r_walk_row_max", "walk_col_iters"),
    ("for (int p0 = 0; p0 < wn", "VSD_STAMP(11);", "walk_passes"),
    ("for (int wb = 0; wb <", "for (int p0 = 0; p0 < wn", "row_windows"),
    ("for (int c0 = 0; c0 <", "for (int wb = 0; wb <", "setup_chunks"),
    ("for (int claimed = 0;; claimed = 1)", "int cnt = 0;", "claim_iters"),
    ("for (int t = sp, it = 0;", "if constexpr (COST == kCostRender) return;", "tile_iters"),
    ("// 3. per-pixel distances", "// step cost: the certified", "pix_compact_rows"),
    ("for (int i = lane; i < npix; i += 64)", "VSD_STAMP(4);", "pix_iters"),
    ("func", "r_raster", "slow"),
    ("func", "region_min8", "zero"),
    ("func", "region_covered", "zero"),
]
# Blocks outside their loop's usual path: their own counters
BLOCK_COUNTERS = {"exact": "exact_ballots", "cull": "zero", "slow_raster": "slow_chunks"}
_RANGES = {}


def _lines(path):
  with open(path) as f:
    return f.read().split("\n")


def _func_range(lines, name):
  """[first, last] 1-based lines of device function `name` (its signature line
  to the first later line that is a lone closing brace)."""
  pat = re.compile(r"^(?:template <.*>\s*)?(?:__device__|__global__).*[ *]%s\(" % re.escape(name))
  for i, l in enumerate(lines):
    if pat.search(l) or (l.startswith("__device__") and (" %s(" % name) in l):
      for j in range(i, len(lines)):
        if lines[j] == "}":
          return i + 1, j + 1
  return None


def _region(lines, start, stop):
  a = next(i for i, l in enumerate(lines) if start in l)
  b = next(i for i in range(a + 1, len(lines)) if stop in lines[i])
  return a + 1, b  # [start line, line before stop]


def ranges():
  if _RANGES:
    return _RANGES
  src = {os.path.basename(p): _lines(p) for p in (SRC, os.path.join(os.path.dirname(SRC),
                                                                      "raster.h"))}
  ph, lp = [], []
  for fname, lines in src.items():
    for name, phase in FUNCS.items():
      r = _func_range(lines, name)
      if r:
        ph.append((fname, r[0], r[1], phase))
  k = src["kern_vsd.hip"]
  reg = [("kern_vsd.hip",) + _region(k, a, b) + (p,) for a, b, p in REGIONS]
  r = src["raster.h"]
  big = "if (__builtin_expect(__builtin_amdgcn_ballot_w64(!t.small) != 0, 0)) {"
  i0 = next(i for i, l in enumerate(r) if big in l)
  i1 = next(i for i in range(i0 + 1, len(r)) if big in r[i])
  reg += [("raster.h", i0 + 1, _region(r[i0:], big, "const RVtx b = neg ? c0 : b0")[1] + i0, "large"),
          ("raster.h", i1 + 1, _region(r[i1:], big, "const RVtx s[3]")[1] + i1, "large"),
          # r_raster's int64 edges (triangles of >= 128 px extent)
          ("raster.h",) + _region(r, "const int64_t py = 256 * (int64_t)row + 128;",
                                  "// Row items (the k_vsd fast path)") + ("large",)]
  _RANGES["phases"] = reg + ph  # k_vsd regions first (lambdas inside k_vsd), then functions
  for a, b, name in LOOP_REGIONS:
    if a == "func":
      for fname, lines in src.items():
        r = _func_range(lines, b)
        if r:
          lp.append((fname, r[0], r[1], name))
    else:
      lp.append(("kern_vsd.hip",) + _region(k, a, b) + (name,))
  _RANGES["loops"] = lp
  return _RANGES


def phase_of(loc):
  if loc is None:
    return "?"
  f, line = loc
  for pf, a, b, name in ranges()["phases"]:
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


# Small prologue / epilogue loops: fixed trips per tuple (anchor region, trips)
CONST_LOOPS = [
    ("for (int k = 0; k < a.n_tau; ++k) fast", "divide = a.normalized && !fast;", 8 * 10.0),
    ("for (int i = tid; i < 2 * kTileStride * kTileH", "__syncthreads();", 8 * 17.0),
    ("// 4. workgroup reduction", "hipError_t read_vsd_stats", 10.0),  # tid 0: n_tau
]
CONST_FUNCS = {"step_threshold": 4.0}  # wave 0: the ulp walk


def _votes(b):
  """The LOOP_REGIONS entry holding most of block b's instruction lines."""
  votes = collections.Counter()
  for _, loc in b["insts"]:
    if not loc:
      continue
    for f, a0, a1, name in ranges()["loops"]:
      if loc[0] == f and a0 <= loc[1] <= a1:
        votes[name] += 1
        break
  return votes.most_common(1)[0][0] if votes else None


def loop_counter(blocks, header):
  """Counter of a loop: the LOOP_REGIONS entry of its header block (r_raster
  loops: rows when the enclosing loop is the set-up chunk loop, columns
  otherwise), a fixed trip count (float) for the small prologue / epilogue
  loops, or None."""
  by = {b["label"]: b for b in blocks}
  b = by.get(header)
  if b is None:
    return None
  name = _votes(b)
  par = b["parents"][-1] if b["parents"] else None
  if name is None:
    src = _lines(SRC)
    for a0, z, trips in CONST_LOOPS:
      r0, r1 = _region(src, a0, z)
      if any(loc and loc[0] == "kern_vsd.hip" and r0 <= loc[1] <= r1 for _, loc in b["insts"]):
        return trips
    for fn, trips in CONST_FUNCS.items():
      r = _func_range(src, fn)
      if r and any(loc and loc[0] == "kern_vsd.hip" and r[0] <= loc[1] <= r[1]
                   for _, loc in b["insts"]):
        return trips
    if any(loc and loc[0].startswith("amd_hip_atomic") for _, loc in b["insts"]):
      return 8.0  # the CAS loop of a lane-0 atomic: once per wave
    # a header without lines of its own (r_raster's small-triangle row loop)
    if par in by and _votes(by[par]) == "setup_chunks":
      kids = [c for c in blocks if c["loop"] == c["label"] and c["parents"] and
              c["parents"][-1] == header]
      if any(_votes(c) == "slow" for c in kids):
        return "slow_rows"
    return None
  if name == "slow":
    name = "slow_rows" if par in by and _votes(by[par]) == "setup_chunks" else "slow_col_iters"
  return name


def block_rare(b):
  """Blocks of the IEEE division fall-back of rcp_rn (inputs outside the
  normal range): not executed on the bench."""
  if any(op.startswith(("v_div_fmas", "v_div_scale", "v_div_fixup")) for op, _ in b["insts"]):
    return True
  locs = [loc for _, loc in b["insts"] if loc]
  rcp = _func_range(_lines(os.path.join(os.path.dirname(SRC), "raster.h")), "rcp_rn")
  # `return ok ? r : 1.0f / x` alone (the ballot-guarded IEEE branch)
  return bool(locs) and rcp is not None and all(
      l[0] == "raster.h" and l[1] == rcp[1] - 2 for l in locs)


def _fine(loc):
  """Lines of the float64 per-pixel sequence (dist_of, sqrt_depth, visib19t,
  vsd_exact_px): in k_vsd's step-cost pixel loop only the exact path uses them."""
  if not loc or loc[0] != "kern_vsd.hip":
    return None
  for f, a0, a1, name in ranges()["phases"]:
    if f == "kern_vsd.hip" and a0 <= loc[1] <= a1:
      break
  src = _lines(SRC)
  for fn in ("sqrt_depth", "dist_of", "visib19t", "vsd_exact_px"):
    r = _func_range(src, fn)
    if r and r[0] <= loc[1] <= r[1]:
      return "pixel_exact"
  return None


HELPERS = ("lib", "?", "rcp")  # lines of shared helpers: counted in the calling block's phase


def block_phase(b, fallback="?"):
  """Majority phase of a block's instructions, helper / compiler lines aside."""
  c = collections.Counter()
  for _, loc in b["insts"]:
    ph = phase_of(loc)
    if ph not in HELPERS and not ph.startswith("other"):
      c[ph] += 1
  return c.most_common(1)[0][0] if c else fallback


def loop_phase(blocks, header):
  """Majority phase of the instructions of a loop's own blocks (helpers aside)."""
  cnt = collections.Counter()
  for b in blocks:
    if b["loop"] == header:
      for op, loc in b["insts"]:
        ph = phase_of(loc)
        if ph not in HELPERS and not ph.startswith("other"):
          cnt[ph] += 1
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
  counts = {}
  if a.counts:
    cj = json.load(open(a.counts))
    counts = dict(cj["wave"])
    counts["zero"] = 0.0
    counts["<top>"] = 8.0  # once per wave
  loop_ctr = {key: loop_counter(blocks, key) for key in loops if key != "<top>"}
  loop_ctr["<top>"] = "<top>"
  dyn = collections.defaultdict(collections.Counter)
  if counts:
    claim_taken = counts["claim_iters"] - counts["tile_iters"]  # iterations past the break
    lphase = {key: (loop_phase(blocks, key) if key != "<top>" else "prologue") for key in loops}
    per_loop_dyn = collections.Counter()
    for b in blocks:
      key = b["loop"] or "<top>"
      name = loop_ctr.get(key)
      major = block_phase(b, lphase.get(key, "?"))
      lines = {phase_of(loc) for _, loc in b["insts"]}
      if block_rare(b) or major in ("cull", "large"):
        name = "zero"
      elif name == "pix_iters" and lines & {"exact"} or (name == "pix_iters" and "pixel_exact"
                                                          in {_fine(loc) for _, loc in b["insts"]}):
        name = "exact_ballots"  # the float64 sequence: the filter's re-runs (and !filter)
      elif major == "slow_raster" and not str(name).startswith("slow"):
        name = "slow_chunks"
      elif name == "claim_iters" and b["label"] != key:
        name = claim_taken  # everything after the claim and its break test
      trip = name if isinstance(name, float) else counts.get(name)
      if trip is None:
        print("  no counter for block %s (loop %s, %s): %d instructions" % (
            b["label"], key, name, len(b["insts"])))
        continue
      for op, loc in b["insts"]:
        ph = phase_of(loc)
        if ph in HELPERS or ph.startswith("other"):
          ph = major  # helper / compiler lines: the block's phase
        dyn[ph][iclass(op)] += trip
        if iclass(op) == "VALU":
          per_loop_dyn[key] += trip
  rows = []
  for key, info in sorted(loops.items(), key=lambda kv: (kv[1]["depth"], kv[0])):
    c = per_loop[key]
    ph = loop_phase(blocks, key) if key != "<top>" else "prologue/epilogue"
    v = sum(n for (p, cl), n in c.items() if cl == "VALU")
    s = sum(n for (p, cl), n in c.items() if cl == "SALU")
    l = sum(n for (p, cl), n in c.items() if cl == "LDS")
    lc = loop_ctr.get(key)
    trip = (lc if isinstance(lc, float) else counts.get(lc)) if counts else None
    rows.append({"loop": key, "depth": info["depth"], "parents": info["parents"], "phase": ph,
                 "blocks": info["blocks"], "valu": v, "salu": s, "lds": l, "trip_per_tuple": trip})
    print("%-10s d%d %-18s blocks %3d  VALU %4d SALU %4d LDS %3d  %-16s%s" % (
        key, info["depth"], ph, info["blocks"], v, s, l, loop_ctr.get(key),
        "" if trip is None else "  trips/tuple %.1f" % trip))
  if counts:
    print("\ndynamic estimate per tuple (each block's static count x its loop's wave-level trips):")
    tot = collections.Counter()
    for p, c in sorted(dyn.items(), key=lambda kv: -kv[1]["VALU"]):
      tot.update(c)
      print("  %-18s VALU %9.0f  SALU %9.0f  LDS %8.0f" % (p, c["VALU"], c["SALU"], c["LDS"]))
    print("  %-18s VALU %9.0f  SALU %9.0f  LDS %8.0f" % ("total", tot["VALU"], tot["SALU"],
                                                        tot["LDS"]))
    print("\nVALU per tuple by loop:")
    for key, v in per_loop_dyn.most_common(12):
      lc = loop_ctr.get(key)
      print("  %-10s %-18s %9.0f" % (key, lc if isinstance(lc, str) else "fixed x%g" % lc, v))
  if a.json:
    with open(a.json, "w") as f:
      json.dump({"kernel": a.kernel, "static_total": total, "loops": rows,
                 "dynamic_per_tuple": {p: dict(c) for p, c in dyn.items()}}, f, indent=1)


if __name__ == "__main__":
  main()
