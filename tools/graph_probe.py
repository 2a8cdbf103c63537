"""Probe: capture one bench step (k_vsd + MSSD + MSPD launches through the
C-ABI on torch's stream) into a HIP graph and replay it; compares the graph's
outputs with eager ones and times both. Diagnostics only.

    python tools/graph_probe.py
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.argv += ["--no-cpu-baseline"]

import torch  # noqa: E402

import bench  # noqa: E402
from bop_toolkit_amd.batch import BatchEvaluator  # noqa: E402


def main():
  args = bench.parse()
  ev = BatchEvaluator(0)
  objs = bench.build_objects(ev, args, torch)
  n, d = bench.build_workload(ev, objs, args, 0, torch)
  o_v = torch.empty((n, bench.N_TAU), dtype=torch.float64, device=ev.device)
  o_s = torch.empty(n, dtype=torch.float64, device=ev.device)
  o_p = torch.empty(n, dtype=torch.float64, device=ev.device)

  def step():
    ev.vsd(d["slots"], d["pose_est"], d["pose_gt"], d["frame_idx"], d["frames"], d["cam"],
           bench.DELTA, bench.TAUS, d["diameters"], out=o_v)
    ev.mssd(d["slots"], d["pose_est"], d["pose_gt"], out=o_s)
    ev.mspd(d["slots"], d["pose_est"], d["pose_gt"], d["K"], out=o_p)

  step()
  torch.cuda.synchronize()
  ref = [o_v.clone(), o_s.clone(), o_p.clone()]
  s = torch.cuda.Stream()
  s.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(s):
    step()
  torch.cuda.current_stream().wait_stream(s)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    step()
  for o in (o_v, o_s, o_p):
    o.zero_()
  g.replay()
  torch.cuda.synchronize()
  same = all(torch.equal(a, b) for a, b in zip(ref, (o_v, o_s, o_p)))
  print("graph outputs identical:", same, flush=True)
  for name, fn in (("eager", step), ("graph", g.replay)) * 2:
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
      fn()
    torch.cuda.synchronize()
    print(name, "%.3f ms/step" % ((time.perf_counter() - t0) / 10 * 1e3), flush=True)


if __name__ == "__main__":
  main()
