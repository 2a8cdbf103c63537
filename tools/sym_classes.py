"""MSSD / MSPD kernel time per symmetry class of the bench objects (where
k_sym_error's time goes). Builds the configs[3] objects as bench.py does, then
times ev.mssd / ev.mspd on --n tuples of each object alone (random GT poses,
perturbed estimates, YCB-V K), events on torch's stream, best of --reps.

    python tools/sym_classes.py [--n 5000] [--reps 5]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--n", type=int, default=5000)
  ap.add_argument("--reps", type=int, default=5)
  a, rest = ap.parse_known_args()
  sys.argv = [sys.argv[0]] + rest
  import torch

  import bench
  from bop_toolkit_amd import synth
  from bop_toolkit_amd.batch import BatchEvaluator
  args = bench.parse()
  ev = BatchEvaluator(0)
  objs = bench.build_objects(ev, args, torch)
  rng = np.random.default_rng(5)
  d = ev.device
  T = lambda x, dt: torch.as_tensor(np.ascontiguousarray(x), dtype=dt, device=d)
  out = []
  seen = set()
  for o, ob in enumerate(objs):
    S = len(ob["syms"])
    if S in seen:
      continue
    seen.add(S)
    Rg, tg = synth.gt_poses(rng, a.n)
    Re, te = synth.perturb(rng, Rg, tg)
    pe = T(np.concatenate([Re.reshape(a.n, 9), te], 1), torch.float64)
    pg = T(np.concatenate([Rg.reshape(a.n, 9), tg], 1), torch.float64)
    K = T(np.tile(synth.YCBV_K.reshape(9), (a.n, 1)), torch.float64)
    slots = ev.slots(np.full(a.n, o, np.int32))
    row = {"object": o, "S": S, "tuples": a.n}
    for name, fn in (("mssd", lambda: ev.mssd(slots, pe, pg)),
                     ("mspd", lambda: ev.mspd(slots, pe, pg, K))):
      fn()
      best = float("inf")
      for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
      row[name + "_ms"] = round(best, 4)
      row[name + "_us_per_1k"] = round(1000.0 * best / a.n * 1000.0, 2)
    out.append(row)
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
  main()
