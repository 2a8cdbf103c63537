#!/usr/bin/env python
"""Latency of the drop-in per-tuple API (what an unmodified reference loop
calls): pose_error.vsd with the HIP renderer (one 640x480 frame uploaded per
call), mssd, mspd, add, adi on a 5k-vertex object. Needs a GPU.

    python tools/percall_bench.py [--calls 200]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--calls", type=int, default=200)
  a = ap.parse_args()
  from bop_toolkit_amd import misc, pose_error, synth
  from bop_toolkit_amd.renderer import create_renderer
  rng = np.random.default_rng(5)
  pts, faces = synth.superellipsoid(50, 100, (60.0, 45.0, 75.0), 0.7)
  info = synth.models_info_entry(pts, 8)
  syms = misc.get_symmetry_transformations(info, 0.01)
  K = synth.YCBV_K
  ren = create_renderer(640, 480, "hip", mode="depth")
  ren.add_object_arrays(1, pts, faces)
  Rg, tg = synth.gt_poses(rng, a.calls)
  Re, te = synth.perturb(rng, Rg, tg)
  depth = ren.render_object(1, Rg[0], tg[0].reshape(3, 1), K[0, 0], K[1, 1], K[0, 2], K[1, 2])
  depth = np.where(depth["depth"] > 0, depth["depth"] + 2.0, 1500.0).astype(np.float32)
  taus = list(np.arange(0.05, 0.51, 0.05))
  out = {}
  fns = {
      "vsd": lambda i: pose_error.vsd(Re[i], te[i].reshape(3, 1), Rg[i], tg[i].reshape(3, 1),
                                      depth, K, 15, taus, True, info["diameter"], ren, 1),
      "mssd": lambda i: pose_error.mssd(Re[i], te[i].reshape(3, 1), Rg[i], tg[i].reshape(3, 1),
                                        pts, syms),
      "mspd": lambda i: pose_error.mspd(Re[i], te[i].reshape(3, 1), Rg[i], tg[i].reshape(3, 1),
                                        K, pts, syms),
      "add": lambda i: pose_error.add(Re[i], te[i].reshape(3, 1), Rg[i], tg[i].reshape(3, 1), pts),
      "adi": lambda i: pose_error.adi(Re[i], te[i].reshape(3, 1), Rg[i], tg[i].reshape(3, 1), pts)}
  for name, fn in fns.items():
    for i in range(5):
      fn(i)
    t = time.perf_counter()
    for i in range(a.calls):
      fn(i)
    out[name + "_ms_per_call"] = round((time.perf_counter() - t) / a.calls * 1e3, 4)
  print(json.dumps({"what": "drop-in per-call latency (one tuple per call, host in/out, "
                            "5k-vertex object, S=8, 640x480)", "calls": a.calls, **out}))


if __name__ == "__main__":
  main()
