"""Device depth-PNG decode time against batch size (frames per
bopx_png_decode_dev launch): is k_png_inflate latency- or throughput-bound?
One wave per stream, so a batch's time stays one stream's latency until the
chip's wave slots are full, then grows with the batch. 512 distinct
Pillow-written 640x480 frames (like tools/png_bench.py) are repeated to make
the larger batches. Prints one JSON line (decode = upload + kernels + status
readback, per DepthDecoder.load; pack = host threads).

    python tools/png_occupancy.py [--sizes 512,1024,...]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--sizes", default="256,512,1024,2048,3072,4096,5120,6144,8192,12288")
  ap.add_argument("--reps", type=int, default=2)
  a = ap.parse_args()
  import torch
  from PIL import Image

  from bop_toolkit_amd import depth_gpu
  rng = np.random.default_rng(1)
  tmp = tempfile.mkdtemp(prefix="pngo_", dir=os.environ.get("TMPDIR", "/tmp"))
  H, W = 480, 640
  yy, xx = np.mgrid[0:H, 0:W]
  paths = []
  for k in range(512):
    d = 16000 + 2000 * np.sin(xx / (40.0 + k % 7)) * np.cos(yy / 31.0)
    cx, cy = 100 + (k * 37) % (W - 200), 80 + (k * 53) % (H - 160)
    d[cy - 60:cy + 60, cx - 80:cx + 80] = 9000 + 30 * np.sin(xx[cy - 60:cy + 60, cx - 80:cx + 80])
    d = d + rng.normal(0, 20, d.shape)
    d[rng.random(d.shape) < 0.1] = 0
    p = os.path.join(tmp, "%06d.png" % k)
    Image.fromarray(np.clip(np.round(d), 0, 65535).astype(np.uint16)).save(p)
    paths.append(p)
  dec = depth_gpu.DepthDecoder(0)
  res = []
  for n in [int(x) for x in a.sizes.split(",")]:
    ps = [paths[i % len(paths)] for i in range(n)]
    best = None
    for r in range(a.reps + 1):
      for k in depth_gpu.STATS:
        depth_gpu.STATS[k] = 0 if k in ("calls", "frames") else 0.0
      f = dec.load(ps, [0.1] * n, H, W, torch)
      torch.cuda.synchronize()
      assert dec.last_host == 0
      del f
      if (r or a.reps == 0) and (best is None or depth_gpu.STATS["decode_s"] < best["decode_s"]):
        best = dict(depth_gpu.STATS)
    res.append({"frames": n, "decode_ms": round(1e3 * best["decode_s"], 2),
                "pack_ms": round(1e3 * best["pack_s"], 2),
                "decode_us_per_frame": round(1e6 * best["decode_s"] / n, 2)})
    print(json.dumps(res[-1]), file=sys.stderr, flush=True)
  print(json.dumps({"what": "depth PNG decode vs batch size (DepthDecoder.load, best of %d)"
                    % a.reps, "runs": res}))


if __name__ == "__main__":
  main()
