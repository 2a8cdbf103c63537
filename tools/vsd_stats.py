"""Workload counters of one k_vsd launch on the bench workload (diagnostics).

    BOPX_VSD_ABLATE=4 python tools/vsd_stats.py [--tuples N]   # counters
    BOPX_VSD_ABLATE=8 python tools/vsd_stats.py [--tuples N]   # phase clocks

Uses the -DBOPX_VSD_DIAG=1 build (make diag), not the product library.
"""
import ctypes
import os
import sys

os.environ.setdefault("BOPX_VSD_ABLATE", "4")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
# counters and clocks exist only in the diagnostic build of the library
if "BOPX_LIB" not in os.environ:
  import subprocess
  subprocess.run(["make", "-s", "-C", os.path.join(REPO, "bop_toolkit_amd", "csrc"), "diag"],
                 check=True)
  os.environ["BOPX_LIB"] = os.path.join(REPO, "bop_toolkit_amd", "lib", "diag", "libbopx_diag.so")
sys.argv += [] if "--tuples" in sys.argv else ["--tuples", "1200"]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from bop_toolkit_amd.batch import BatchEvaluator  # noqa: E402


def main():
  args = bench.parse()
  ev = BatchEvaluator(0)
  objs = bench.build_objects(ev, args, torch)
  n, d = bench.build_workload(ev, objs, args, 0, 1, torch)
  fn = ev.ctx.lib.bopx_debug_vsd_stats
  fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
  st = (ctypes.c_ulonglong * 48)()
  fn(ev.ctx.h, st, 1)
  ev.vsd(d["slots"], d["pose_est"], d["pose_gt"], d["frame_idx"], d["frames"], d["cam"],
         bench.DELTA, bench.TAUS, d["diameters"])
  torch.cuda.synchronize()
  fn(ev.ctx.h, st, 1)
  names = ["tiles", "meshlet_entries", "tri_setups", "bbox_iters", "rows",
           "fragments", "covered_px", "row_passes", "pass_max_w_sum", "culled_entries",
           "slow_tris", "slow_bbox_px", "slow_waves", "large_tris", "exact_px"]
  for i, k in enumerate(names):
    print("%-20s total %14d  per tuple %12.1f" % (k, st[i], st[i] / n))
  ph = ["clear+coeffs", "list", "raster work", "raster barrier", "pixel work",
        "pixel barrier", "pre-loop", "epilogue", "r:stage", "r:compact", "r:setup", "r:walk",
        "r:claim", "r:vload", "r:occl"]
  tot = sum(st[16 + i] for i in range(16))
  for i, k in enumerate(ph):
    print("phase %-16s %6.1f %%  (%.3g cycles/wave-tuple)" % (k, 100.0 * st[16 + i] / max(1, tot),
                                                           st[16 + i] / n / 8))
  roi = bench.roi_pixels(objs, d["host"]["obj"], [d["host"]["pe"], d["host"]["pg"]],
                         bench.synth_K() if hasattr(bench, "synth_K") else __import__(
                             "bop_toolkit_amd.synth", fromlist=["YCBV_K"]).YCBV_K)
  print("bbox-corner ROI mean px %.0f" % np.mean(roi))
  wave = ["claim_iters", "setup_chunks", "row_windows", "walk_passes", "walk_col_iters",
          "pix_compact_rows", "pix_iters", "exact_ballots", "slow_col_iters", "slow_rows",
          "list_calls", "tile_iters", "slow_chunks"]
  for i, k in enumerate(wave):
    print("wave %-18s total %14d  per tuple %12.2f" % (k, st[32 + i], st[32 + i] / n))
  out = os.environ.get("BOPX_VSD_STATS_JSON")
  if out:
    import json
    with open(out, "w") as f:
      json.dump({"tuples": n, "workload": bench.workload_key(args, n),
                 "stats": {k: st[i] / n for i, k in enumerate(names)},
                 "wave": {k: st[32 + i] / n for i, k in enumerate(wave)},
                 "phase_cycles_per_wave_tuple": {k: st[16 + i] / n / 8 for i, k in enumerate(ph)}},
                f, indent=1)


if __name__ == "__main__":
  main()
