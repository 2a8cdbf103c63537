"""Depth PNG decode throughput: host decoder (libbopx_io.so, threads) vs the
device decoder (depth_gpu.DepthDecoder: pack on host threads + one DMA +
kern_png.hip). Frames like the e2e set: a smooth scene + N(0, 2 mm) noise at
depth_scale 0.1 + 10 % holes, written by Pillow. Prints one JSON line.

    python tools/png_bench.py [--frames 512] [--reps 3]
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
  ap.add_argument("--frames", type=int, default=512)
  ap.add_argument("--reps", type=int, default=3)
  ap.add_argument("--h", type=int, default=480)
  ap.add_argument("--w", type=int, default=640)
  a = ap.parse_args()
  import torch
  from PIL import Image

  from bop_toolkit_amd import depth_gpu, inout
  rng = np.random.default_rng(1)
  tmp = tempfile.mkdtemp(prefix="pngb_", dir=os.environ.get("TMPDIR", "/tmp"))
  yy, xx = np.mgrid[0:a.h, 0:a.w]
  paths = []
  for k in range(a.frames):
    d = 16000 + 2000 * np.sin(xx / (40.0 + k % 7)) * np.cos(yy / 31.0)
    cx, cy = 100 + (k * 37) % (a.w - 200), 80 + (k * 53) % (a.h - 160)
    d[cy - 60:cy + 60, cx - 80:cx + 80] = 9000 + 30 * np.sin(xx[cy - 60:cy + 60, cx - 80:cx + 80])
    d = d + rng.normal(0, 20, d.shape)
    d[rng.random(d.shape) < 0.1] = 0
    p = os.path.join(tmp, "%06d.png" % k)
    Image.fromarray(np.clip(np.round(d), 0, 65535).astype(np.uint16)).save(p)
    paths.append(p)
  scales = [0.1] * a.frames
  mb = sum(os.path.getsize(p) for p in paths) / 1e6
  dec = depth_gpu.DepthDecoder(0)
  dev = torch.device("cuda", 0)
  out = np.empty((a.frames, a.h, a.w), np.float32)
  host, gpu, kern = [], [], []
  for r in range(a.reps + 1):
    t = time.perf_counter()
    inout.load_depths(paths, scales=scales, out=out)
    host.append(time.perf_counter() - t)
    torch.cuda.synchronize()
    t = time.perf_counter()
    f = dec.load(paths, scales, a.h, a.w, torch)
    torch.cuda.synchronize()
    gpu.append(time.perf_counter() - t)
    if r == 0:
      assert dec.last_host == 0
      assert np.array_equal(f.cpu().numpy().view(np.uint32), out.view(np.uint32))
  # kernels alone: the packed stream resident, decode launched twice
  buf, need, z_off, z_len, st = depth_gpu.pack(paths, a.h, a.w, lambda nb: np.zeros(nb, np.uint8))
  z = torch.from_numpy(buf[:need]).to(dev)
  off, ln = torch.from_numpy(z_off).to(dev), torch.from_numpy(z_len).to(dev)
  stride = depth_gpu.raw_stride_of(a.h, a.w)
  raw = torch.empty(a.frames * stride, dtype=torch.uint8, device=dev)
  fr = torch.empty((a.frames, a.h, a.w), dtype=torch.float32, device=dev)
  stat = torch.empty(2 * a.frames, dtype=torch.int32, device=dev)
  import ctypes
  s = torch.cuda.current_stream(dev)
  for r in range(a.reps + 1):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    dec.ctx.call("bopx_png_decode_dev", a.frames, z.data_ptr(), off.data_ptr(), ln.data_ptr(),
                 a.h, a.w, None, raw.data_ptr(), stride, fr.data_ptr(), stat.data_ptr(),
                 ctypes.c_void_p(s.cuda_stream))
    e1.record()
    torch.cuda.synchronize()
    kern.append(e0.elapsed_time(e1) / 1e3)
  best = lambda v: min(v[1:])
  print(json.dumps({
      "frames": a.frames, "size": [a.w, a.h], "png_mb": round(mb, 1),
      "host_s": round(best(host), 4), "host_threads": min(16, os.cpu_count() or 1),
      "device_s": round(best(gpu), 4), "device_kernels_s": round(best(kern), 4),
      "host_fps": round(a.frames / best(host), 1), "device_fps": round(a.frames / best(gpu), 1),
      "kernel_fps": round(a.frames / best(kern), 1),
      "kernel_png_gb_s": round(mb / 1e3 / best(kern), 2)}), flush=True)


if __name__ == "__main__":
  main()
