#!/usr/bin/env python
"""Batch-size sweep of the k_vsd tile-parallel mode: wall time per
bopx_vsd_batch call (one 640x480 frame, 5k-vertex object, 10 taus) for batch
sizes 1..512. Run once per BOPX_VSD_SPLIT setting (read once per process):

    BOPX_VSD_SPLIT=1 python tools/split_sweep.py    # one workgroup per tuple
    python tools/split_sweep.py [n1,n2,...]         # automatic split
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
  from bop_toolkit_amd import _lib, synth
  from bop_toolkit_amd._lib import _d, _f, _i32, ptr
  rng = np.random.default_rng(3)
  pts, faces = synth.superellipsoid(50, 100, (60.0, 45.0, 75.0), 0.7)
  K = synth.YCBV_K
  sizes = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else
                            "1,4,16,32,64,128,192,255,256,512".split(","))]
  nmax, W, H = max(sizes), 640, 480
  Rg, tg = synth.gt_poses(rng, nmax)
  Re, te = synth.perturb(rng, Rg, tg)
  ctx = _lib.Context(0)
  ctx.add_object(1, pts, faces)
  frame = np.round(rng.uniform(400.0, 1400.0, (1, H, W))).astype(np.float32)
  taus = np.arange(0.05, 0.51, 0.05)
  pe = np.concatenate([Re.reshape(nmax, 9), te], 1)
  pg = np.concatenate([Rg.reshape(nmax, 9), tg], 1)
  cam = np.array([[K[0, 0], K[1, 1], K[0, 2], K[1, 2]]], np.float64)
  res = {}
  for n in sizes:
    ids = np.ones(n, np.int32)
    fi = np.zeros(n, np.int32)
    dia = np.full(n, 180.0)
    out = np.empty((n, len(taus)))
    p_e, p_g = pe[:n].copy(), pg[:n].copy()

    def call():
      ctx.call("bopx_vsd_batch", n, ptr(ids, _i32), ptr(p_e, _d), ptr(p_g, _d), ptr(fi, _i32),
               ptr(frame, _f), 1, W, H, ptr(cam, _d), 15.0, 0, ptr(taus, _d), len(taus), 1,
               ptr(dia, _d), 0, ptr(out, _d))
    for _ in range(3):
      call()
    ts = []
    for _ in range(30):
      t = time.perf_counter()
      call()
      ts.append(time.perf_counter() - t)
    res[n] = round(float(np.median(ts)) * 1e3, 4)
  ctx.close()
  print(json.dumps({"split": os.environ.get("BOPX_VSD_SPLIT", "auto"), "ms_per_call": res}))


if __name__ == "__main__":
  main()
