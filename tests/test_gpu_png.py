"""Depth PNG decode on the GPU (kern_png.hip, bopx_png_decode_dev) vs the host
decoder (libbopx_io.so, itself pinned to Pillow in test_depth_png.py).

The reference reads test depth with inout.load_depth (bop_toolkit_lib/
inout.py:39-46) and scales it in float32 (scripts/eval_calc_errors.py:242-243).
The device frames must equal the host decoder's bit for bit for every zlib
stream an encoder can produce (levels 0-9, window sizes, the FILTERED /
HUFFMAN_ONLY / RLE / FIXED strategies, stored blocks, IDAT split anywhere)
and every PNG row filter, and a stream the device rejects must fall back to
the host path, which then gives its own result or error.
"""
import ctypes
import os
import zlib

import numpy as np
import pytest
from PIL import Image

from test_depth_png import _depth, _filter_rows, far_match_stream, png_from_zlib, write_png16

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dec():
  if not torch.cuda.is_available():
    pytest.skip("no GPU")
  from bop_toolkit_amd import depth_gpu
  return depth_gpu.DepthDecoder(0)


def _host(paths, scales, h, w):
  from bop_toolkit_amd import inout
  out = np.empty((len(paths), h, w), np.float32)
  inout.load_depths(paths, scales=scales, out=out)
  return out


def _zvariant(k):
  """zlib stream writers: (level, wbits, memLevel, strategy)."""
  S = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED]
  level = [0, 1, 6, 9, 3, 9, 6][k % 7]
  wbits = [15, 9, 12, 15, 10, 15][k % 6]
  strat = S[k % 5]
  mem = [8, 9, 1, 5][k % 4]

  def comp(raw):
    c = zlib.compressobj(level, zlib.DEFLATED, wbits, mem, strat)
    return c.compress(raw) + c.flush()
  return comp


def _image(rng, kind, h, w):
  if kind == 0:
    return _depth(rng, h, w)
  if kind == 1:  # sensor-like noise: literal-heavy streams
    return np.clip(rng.normal(16000, 20, (h, w)), 0, 65535).astype(np.uint16)
  if kind == 2:  # constant: long distance-2 matches
    return np.full((h, w), 1234, np.uint16)
  if kind == 3:
    return np.zeros((h, w), np.uint16)
  if kind == 4:  # full range random
    return rng.integers(0, 65536, (h, w), dtype=np.uint16)
  yy, xx = np.mgrid[0:h, 0:w]  # gradient with holes
  d = (500 + 3 * xx + 7 * yy).astype(np.uint16)
  d[(xx // 5 + yy // 3) % 4 == 0] = 0
  return d


# (441, 1): one-pixel rows (3 bytes), where a lane's first groups start before
# the frame (the 3,000-stream fuzz at seed 6006 found these on the host path)
@pytest.mark.parametrize("h,w", [(48, 64), (1, 1), (3, 1000), (37, 41), (2, 4096), (441, 1),
                                 (70, 2)])
def test_gpu_decode_matches_host(tmp_path, dec, h, w):
  rng = np.random.default_rng(h * 7919 + w)
  paths, scales = [], []
  for k in range(42):
    img = _image(rng, k % 6, h, w)
    p = str(tmp_path / ("%03d.png" % k))
    filters = [(0,), (1,), (2,), (3,), (4,), (4, 3, 2, 1, 0), (2, 4)][k % 7]
    write_png16(p, img, filters=filters, compress=_zvariant(k),
                idat_split=[None, 1, 7, 333, 8192][k % 5])
    paths.append(p)
    scales.append([1.0, 0.1, 0.25, 1.0 / 3.0, 10.0][k % 5])
  for k in range(6):  # Pillow's own encoder (adaptive filters)
    p = str(tmp_path / ("pil%d.png" % k))
    Image.fromarray(_image(rng, k, h, w)).save(p, compress_level=[0, 1, 6, 9, 6, 3][k])
    paths.append(p)
    scales.append(0.1)
  got = dec.load(paths, scales, h, w, torch).cpu().numpy()
  assert dec.last_host == 0  # every stream decoded on the device
  assert np.array_equal(got.view(np.uint32), _host(paths, scales, h, w).view(np.uint32))


def test_gpu_decode_full_frames(tmp_path, dec):
  """640x480 frames as the evaluation reads them (Pillow-written, depth_scale
  0.1 like YCB-V), in one batch with IDAT split at 8 KiB."""
  rng = np.random.default_rng(5)
  paths = []
  for k in range(24):
    img = _image(rng, [0, 1, 5][k % 3], 480, 640)
    p = str(tmp_path / ("%06d.png" % k))
    if k % 2:
      Image.fromarray(img).save(p)
    else:
      write_png16(p, img, filters=(4, 2, 1), idat_split=8192)
    paths.append(p)
  scales = [0.1] * len(paths)
  got = dec.load(paths, scales, 480, 640, torch)
  assert got.shape == (24, 480, 640) and got.dtype == torch.float32
  assert dec.last_host == 0
  assert np.array_equal(got.cpu().numpy().view(np.uint32),
                        _host(paths, scales, 480, 640).view(np.uint32))


def test_gpu_decode_far_matches(tmp_path, dec):
  """258-byte matches at distances 4100-4350 (a T-LESS 720-px row is 1,441
  bytes, so a 3-row distance is 4,323): past the 4 KB ring by less than a
  copy's length, so later copy rounds must read the flushed output, not ring
  slots the same copy already rewrote. Decoded on the device (no host
  fallback) and equal to the host decoder."""
  rng = np.random.default_rng(17)
  h, w = 24, 720
  paths = []
  for period in (4100, 4166, 4323, 4350):
    z, _ = far_match_stream(rng, period, h, w)
    p = str(tmp_path / ("far%d.png" % period))
    png_from_zlib(p, w, h, z)
    paths.append(p)
  got = dec.load(paths, None, h, w, torch).cpu().numpy()
  assert dec.last_host == 0
  assert np.array_equal(got.view(np.uint32), _host(paths, None, h, w).view(np.uint32))


def test_gpu_decode_host_rows_final_for_other_streams(tmp_path, dec):
  """A batch with a file only the host decodes (8-bit) and clean ones: the
  frames load() returns are final for a consumer on another stream (the
  scene prefetch hands them to the error kernels' stream)."""
  rng = np.random.default_rng(21)
  h, w = 480, 640
  paths = []
  for k in range(6):
    p = str(tmp_path / ("c%d.png" % k))
    write_png16(p, _image(rng, k % 6, h, w))
    paths.append(p)
  p8 = str(tmp_path / "g8.png")
  Image.fromarray((_image(rng, 0, h, w) % 256).astype(np.uint8)).save(p8)
  paths.insert(3, p8)
  side = torch.cuda.Stream()
  with torch.cuda.stream(side):
    got = dec.load(paths, [0.1] * len(paths), h, w, torch)
  consumer = torch.cuda.Stream()
  with torch.cuda.stream(consumer):
    snap = got.clone()
  consumer.synchronize()
  assert dec.last_host == 1
  assert np.array_equal(snap.cpu().numpy(), _host(paths, [0.1] * len(paths), h, w))


def test_group_prefetch_frames_final_for_consumer(tmp_path):
  """GroupPrefetch submits and finishes groups on its worker thread (whose
  current stream is not the decode stream): every scene's slice is the host
  decode when get() returns, read on a third stream without further sync,
  across several groups and one host-only file."""
  if not torch.cuda.is_available():
    pytest.skip("no GPU")
  from bop_toolkit_amd import depth_gpu
  rng = np.random.default_rng(29)
  h, w = 480, 640
  scenes = {}
  for s in range(5):
    ps = []
    for k in range(3 + s):
      p = str(tmp_path / ("s%d_%d.png" % (s, k)))
      if s == 2 and k == 1:
        Image.fromarray((_image(rng, 0, h, w) % 256).astype(np.uint8)).save(p)
      else:
        write_png16(p, _image(rng, (s + k) % 6, h, w))
      ps.append(p)
    scenes[s] = ps
  items = [(s, (lambda ps=ps: (ps, [0.1] * len(ps)))) for s, ps in scenes.items()]
  stream, consumer = torch.cuda.Stream(), torch.cuda.Stream()
  with depth_gpu.GroupPrefetch(0, items, h, w, torch, stream, consumer, max_frames=7) as g:
    for s, ps in scenes.items():
      fr = g.get(s)
      with torch.cuda.stream(consumer):
        snap = fr.clone()
      consumer.synchronize()
      assert np.array_equal(snap.cpu().numpy(), _host(ps, [0.1] * len(ps), h, w)), s
    assert g.groups >= 3


def test_gpu_decode_rejects_what_the_host_rejects(tmp_path, dec):
  """Mutated zlib streams (valid chunk CRCs, so the packer passes them on):
  a stream the device accepts decodes to the host decoder's frame; any other
  goes to the host path, whose result or error load() reproduces."""
  from bop_toolkit_amd import inout
  rng = np.random.default_rng(9)
  h, w = 24, 40
  base = []
  for k in range(6):
    raw = _filter_rows(_image(rng, k, h, w), (k % 5,))
    base.append(_zvariant(k)(raw))
  paths, good = [], []
  for k in range(120):
    z = bytearray(base[k % 6])
    kind = k % 6
    if kind == 0:  # bit flips anywhere
      for _ in range(1 + k % 3):
        i = int(rng.integers(0, len(z)))
        z[i] ^= 1 << int(rng.integers(0, 8))
    elif kind == 1:  # truncated
      z = z[:int(rng.integers(1, len(z)))]
    elif kind == 2:  # Adler-32 wrong
      z[-1] ^= 0x80
    elif kind == 3:  # trailing bytes after the stream (accepted by zlib / libdeflate)
      z += bytes(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8))
    elif kind == 4:  # header: bad FCHECK / preset dictionary
      z[1] ^= 0x20 if k % 2 else 0x01
    else:  # first block's header bits
      z[2] ^= 1 << int(rng.integers(0, 3))
    p = str(tmp_path / ("m%03d.png" % k))
    png_from_zlib(p, w, h, bytes(z), idat_split=int(rng.integers(1, 64)))
    paths.append(p)
  for k, p in enumerate(paths):
    try:
      want = inout.load_depth(p)
    except Exception as e:  # noqa: BLE001
      with pytest.raises(type(e)):
        dec.load([p], None, h, w, torch)
    else:
      good.append(p)
      assert np.array_equal(dec.load([p], None, h, w, torch).cpu().numpy()[0], want)
  assert len(good) >= 20  # the trailing-bytes cases at least
  # the whole set in one batch: every accepted file identical, and the device
  # took the clean ones itself
  got = dec.load(good, None, h, w, torch).cpu().numpy()
  assert np.array_equal(got, _host(good, None, h, w))


def test_gpu_decode_other_files_go_to_host(tmp_path, dec):
  """8-bit / TIFF / wrong-size files in a batch: host decoder for those,
  device for the rest, one frame array; a wrong size raises ValueError."""
  rng = np.random.default_rng(13)
  h, w = 20, 30
  paths = []
  for k in range(4):
    p = str(tmp_path / ("d%d.png" % k))
    write_png16(p, _image(rng, k, h, w))
    paths.append(p)
  p8 = str(tmp_path / "g8.png")
  Image.fromarray((_image(rng, 0, h, w) % 256).astype(np.uint8)).save(p8)
  ptif = str(tmp_path / "d.tif")
  Image.fromarray(_image(rng, 5, h, w)).save(ptif)
  paths += [p8, ptif]
  scales = [0.5] * len(paths)
  got = dec.load(paths, scales, h, w, torch).cpu().numpy()
  assert dec.last_host == 2
  assert np.array_equal(got, _host(paths, scales, h, w))
  psz = str(tmp_path / "size.png")
  write_png16(psz, _image(rng, 0, h + 1, w))
  with pytest.raises(ValueError):
    dec.load(paths[:2] + [psz], None, h, w, torch)


def test_png_decode_dev_argument_checks(dec):
  """The C-ABI refuses sizes outside the kernel's range and short raw strides
  (nothing launched)."""
  ctx = dec.ctx
  s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
  nul = ctypes.c_void_p(0)
  with pytest.raises(ValueError):
    ctx.call("bopx_png_decode_dev", 1, nul, nul, nul, 10, 4097, nul, nul, 1 << 20, nul, nul, s)
  with pytest.raises(ValueError):
    ctx.call("bopx_png_decode_dev", 1, nul, nul, nul, 10, 10, nul, nul, 256, nul, nul, s)
  ctx.call("bopx_png_decode_dev", 0, nul, nul, nul, 10, 10, nul, nul, 1024, nul, nul, s)
