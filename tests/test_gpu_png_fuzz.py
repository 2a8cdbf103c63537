"""Randomised parity of the GPU depth-PNG decoder (kern_png.hip) against the
host decoder: random frame sizes and contents (depth-like, noise, constant,
gradients with holes, full-range random, sparse objects on zeros), zlib
level / window bits / memLevel / strategy, row filter sequences and IDAT
splits, several batches per run. Every frame must decode on the device
(no host fall-back) and equal the host decoder's bits.

BOPX_PNG_FUZZ=N sets the number of streams (default 96; the round-5 run used
3,000: profiles/r05/png_fuzz3000.txt)."""
import os
import zlib

import numpy as np
import pytest

from test_depth_png import _depth, write_png16

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _host(paths, scales, h, w):
  from bop_toolkit_amd import inout
  out = np.empty((len(paths), h, w), np.float32)
  inout.load_depths(paths, scales=scales, out=out)
  return out


def _content(rng, kind, h, w):
  if kind == 0:
    return _depth(rng, h, w)
  if kind == 1:
    return np.clip(rng.normal(rng.uniform(300, 60000), rng.uniform(1, 200), (h, w)), 0,
                   65535).astype(np.uint16)
  if kind == 2:
    return np.full((h, w), int(rng.integers(0, 65536)), np.uint16)
  if kind == 3:
    yy, xx = np.mgrid[0:h, 0:w]
    d = (int(rng.integers(0, 20000)) + int(rng.integers(-9, 9)) * xx +
         int(rng.integers(-9, 9)) * yy) % 65536
    d = d.astype(np.uint16)
    d[rng.random((h, w)) < rng.uniform(0, 0.5)] = 0
    return d
  if kind == 4:
    return rng.integers(0, 65536, (h, w), dtype=np.uint16)
  d = np.zeros((h, w), np.uint16)  # a few objects on an empty background
  for _ in range(int(rng.integers(0, 6))):
    y0, x0 = int(rng.integers(0, h)), int(rng.integers(0, w))
    y1, x1 = min(h, y0 + int(rng.integers(1, 200))), min(w, x0 + int(rng.integers(1, 200)))
    d[y0:y1, x0:x1] = _depth(rng, y1 - y0, x1 - x0)
  return d


def _compressor(rng):
  level = int(rng.integers(0, 10))
  wbits = int(rng.integers(9, 16))
  mem = int(rng.integers(1, 10))
  strat = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE,
           zlib.Z_FIXED][int(rng.integers(0, 5))]

  def comp(raw):
    c = zlib.compressobj(level, zlib.DEFLATED, wbits, mem, strat)
    return c.compress(raw) + c.flush()
  return comp


def test_gpu_png_fuzz(tmp_path):
  if not torch.cuda.is_available():
    pytest.skip("no GPU")
  from bop_toolkit_amd import depth_gpu
  dec = depth_gpu.DepthDecoder(0)
  n_total = int(os.environ.get("BOPX_PNG_FUZZ", "96"))
  rng = np.random.default_rng(int(os.environ.get("BOPX_PNG_FUZZ_SEED", "1234")))
  done = 0
  batch = 0
  while done < n_total:
    h, w = int(rng.integers(1, 500)), int(rng.integers(1, 700))
    m = min(n_total - done, int(rng.integers(1, 64)))
    paths, scales = [], []
    for k in range(m):
      img = _content(rng, int(rng.integers(0, 6)), h, w)
      nf = int(rng.integers(1, 6))
      filters = tuple(int(x) for x in rng.integers(0, 5, nf))
      split = [None, 1, 7, 333, 8192, int(rng.integers(1, 20000))][int(rng.integers(0, 6))]
      p = str(tmp_path / ("b%d_%d.png" % (batch, k)))
      write_png16(p, img, filters=filters, compress=_compressor(rng), idat_split=split)
      paths.append(p)
      scales.append(float(rng.choice([1.0, 0.1, 0.25, 1.0 / 3.0, 10.0])))
    got = dec.load(paths, scales, h, w, torch).cpu().numpy()
    assert dec.last_host == 0, (batch, h, w)
    want = _host(paths, scales, h, w)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (batch, h, w)
    for p in paths:
      os.remove(p)
    done += m
    batch += 1
