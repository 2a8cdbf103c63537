"""Native depth PNG decoder (include/bopx_io.h, libbopx_io.so) vs Pillow.

The reference reads depth with imageio (inout.py:39-46) and scales it in
float32 (eval_calc_errors.py:242-243); the build's loader must return the same
float32 frames bit for bit. PNGs are written here with a small encoder that
picks every PNG row filter (0-4) and splits IDAT, so each decoder branch runs.
CPU only (no GPU).
"""
import os
import struct
import subprocess
import sys
import zlib

import numpy as np
import pytest
from PIL import Image

from bop_toolkit_amd import inout

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _chunk(typ, body):
  return struct.pack(">I", len(body)) + typ + body + struct.pack(">I", zlib.crc32(typ + body))


def _filter_rows(img, filters):
  """PNG-filter a uint16 image (big-endian, 2 bytes per pixel) row by row."""
  h, w = img.shape
  raw = img.astype(">u2").view(np.uint8).reshape(h, 2 * w).astype(np.int32)
  out = []
  for r in range(h):
    f = filters[r % len(filters)]
    cur = raw[r]
    prev = raw[r - 1] if r else np.zeros_like(cur)
    a = np.concatenate([[0, 0], cur[:-2]])
    c = np.concatenate([[0, 0], prev[:-2]])
    if f == 0:
      pred = np.zeros_like(cur)
    elif f == 1:
      pred = a
    elif f == 2:
      pred = prev
    elif f == 3:
      pred = (a + prev) >> 1
    else:
      p = a + prev - c
      pa, pb, pc = np.abs(p - a), np.abs(p - prev), np.abs(p - c)
      pred = np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, prev, c))
    out.append(bytes([f]) + ((cur - pred) & 0xFF).astype(np.uint8).tobytes())
  return b"".join(out)


def write_png16(path, img, filters=(0, 1, 2, 3, 4), idat_split=None, extra=b"", compress=None):
  """compress: raw scanlines -> zlib stream (default zlib.compress level 6)."""
  h, w = img.shape
  raw = _filter_rows(img, filters)
  data = compress(raw) if compress else zlib.compress(raw, 6)
  png_from_zlib(path, w, h, data, idat_split, extra)


def png_from_zlib(path, w, h, data, idat_split=None, extra=b""):
  """A 16-bit gray PNG around the zlib stream `data` (valid chunk CRCs)."""
  parts = [data] if not idat_split else [data[i:i + idat_split]
                                         for i in range(0, len(data), idat_split)]
  ihdr = struct.pack(">IIBBBBB", w, h, 16, 0, 0, 0, 0)
  with open(path, "wb") as f:
    f.write(b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + extra)
    for p in parts:
      f.write(_chunk(b"IDAT", p))
    f.write(_chunk(b"IEND", b""))


def _pillow(path, scale=None):
  d = np.asarray(Image.open(path)).astype(np.float32)
  if scale is not None:
    d *= scale  # the reference's in-place float32 multiply by a JSON float
  return d


def _depth(rng, h, w):
  yy, xx = np.mgrid[0:h, 0:w]
  d = 900 + 400 * np.sin(xx / 37.0) * np.cos(yy / 23.0) + rng.normal(0, 3, (h, w))
  d = np.clip(d, 0, 65535).astype(np.uint16)
  d[rng.random((h, w)) < 0.1] = 0
  d.flat[:3] = [65535, 1, 0]
  return d


@pytest.mark.parametrize("h,w", [(1, 1), (1, 7), (5, 1), (37, 41), (480, 640)])
@pytest.mark.parametrize("filters", [(0,), (1,), (2,), (3,), (4,), (4, 3, 2, 1, 0)])
def test_filters_and_sizes_match_pillow(tmp_path, h, w, filters):
  rng = np.random.default_rng(h * 1000 + w + 7 * filters[0])
  img = _depth(rng, h, w)
  p = str(tmp_path / "d.png")
  write_png16(p, img, filters=filters, idat_split=4096 if h * w > 1000 else None)
  got = inout.load_depth(p)
  assert got.dtype == np.float32 and got.shape == (h, w)
  assert np.array_equal(got, img.astype(np.float32))
  assert np.array_equal(got, _pillow(p))


def test_batch_scales_out_buffer_and_pillow_saved_files(tmp_path):
  rng = np.random.default_rng(3)
  paths, scales = [], [1.0, 0.1, 0.25, 1.0 / 3.0, 10.0, 0.0001]
  for i, s in enumerate(scales):
    p = str(tmp_path / ("%06d.png" % i))
    img = _depth(rng, 48, 64)
    if i % 2:
      Image.fromarray(img).save(p)  # Pillow's own encoder (adaptive filters)
    else:
      write_png16(p, img, idat_split=1000)
    paths.append(p)
  want = np.stack([_pillow(p, s) for p, s in zip(paths, scales)])
  got_list = inout.load_depths(paths, scales=scales)
  assert all(np.array_equal(g, w) for g, w in zip(got_list, want))
  out = np.full((len(paths), 48, 64), -1, np.float32)
  assert inout.load_depths(paths, scales=scales, out=out, workers=3) is out
  assert np.array_equal(out, want)
  # a non-contiguous / float64 destination still receives the same values
  out64 = np.zeros((len(paths), 48, 64), np.float64)
  inout.load_depths(paths, scales=scales, out=out64)
  assert np.array_equal(out64, want.astype(np.float64))


def test_other_formats_go_through_pillow(tmp_path):
  rng = np.random.default_rng(5)
  img = _depth(rng, 20, 30)
  p8 = str(tmp_path / "g8.png")
  Image.fromarray((img % 256).astype(np.uint8)).save(p8)
  prgb = str(tmp_path / "rgb.png")
  Image.fromarray(np.stack([(img % 256).astype(np.uint8)] * 3, -1)).save(prgb)
  ptif = str(tmp_path / "d.tif")
  Image.fromarray(img).save(ptif)
  for p in (p8, prgb, ptif):
    assert np.array_equal(inout.load_depth(p), _pillow(p))
  got = inout.load_depths([p8, ptif], scales=[0.5, 0.1])
  assert np.array_equal(got[0], _pillow(p8, 0.5)) and np.array_equal(got[1], _pillow(ptif, 0.1))


def test_size_mismatch_and_corrupt_files(tmp_path):
  rng = np.random.default_rng(9)
  p = str(tmp_path / "a.png")
  write_png16(p, _depth(rng, 10, 12))
  with pytest.raises(ValueError, match="expected"):
    inout.load_depths([p], out=np.zeros((1, 12, 10), np.float32))
  # a flipped IDAT byte: the native CRC check rejects it and Pillow decides
  raw = bytearray(open(p, "rb").read())
  idat = raw.index(b"IDAT")
  raw[idat + 10] ^= 0x55
  bad = str(tmp_path / "bad.png")
  open(bad, "wb").write(bytes(raw))
  try:
    want = _pillow(bad)
  except Exception as e:  # noqa: BLE001
    with pytest.raises(type(e)):
      inout.load_depth(bad)
  else:
    assert np.array_equal(inout.load_depth(bad), want)
  trunc = str(tmp_path / "trunc.png")
  open(trunc, "wb").write(bytes(raw[:len(raw) // 2]))
  with pytest.raises(Exception):
    inout.load_depth(trunc)
  with pytest.raises(Exception):
    inout.load_depth(str(tmp_path / "missing.png"))


def test_ancillary_chunk_skipped_and_zlib_backend_identical(tmp_path):
  rng = np.random.default_rng(11)
  img = _depth(rng, 33, 65)
  p = str(tmp_path / "t.png")
  write_png16(p, img, extra=_chunk(b"tEXt", b"Comment\x00bopx"), idat_split=500)
  assert np.array_equal(inout.load_depth(p), _pillow(p))
  code = ("import sys, numpy as np; sys.path.insert(0, %r); from bop_toolkit_amd import inout; "
          "assert inout._io_lib().bopx_io_backend() == 0; "
          "np.save(%r, inout.load_depth(%r))" % (REPO, str(tmp_path / "z.npy"), p))
  env = dict(os.environ, BOPX_IO_ZLIB="1")
  subprocess.check_call([sys.executable, "-c", code], env=env)
  assert np.array_equal(np.load(str(tmp_path / "z.npy")), _pillow(p))


def test_scale_is_one_float32_multiply(tmp_path):
  """depth_scale is applied as float32(sample) * float32(scale) for every scalar
  type — what the reference's `depth *= depth_scale` does with its JSON float
  (and, under its NumPy < 1.24, with a numpy float64 too)."""
  rng = np.random.default_rng(13)
  p = str(tmp_path / "s.png")
  img = _depth(rng, 16, 16)
  write_png16(p, img)
  for s in (0.1, np.float64(0.1), np.float32(0.1), 1.0 / 3.0, 7):
    got = inout.load_depths([p], scales=[s])[0]
    want = img.astype(np.float32) * np.float32(s)
    assert got.dtype == np.float32 and np.array_equal(got, want), s


def test_pack_for_the_device_decoder(tmp_path):
  """bopx_pack_depth_pngs (the host half of the GPU decoder): offsets on
  256-byte boundaries from the file sizes, each file's IDAT payloads
  concatenated in place (= the zlib stream), the same per-file checks and
  status codes as the host decoder."""
  from bop_toolkit_amd import depth_gpu
  rng = np.random.default_rng(21)
  paths, streams = [], []
  for i in range(5):
    img = _depth(rng, 30, 40)
    p = str(tmp_path / ("%d.png" % i))
    z = zlib.compress(_filter_rows(img, (i % 5,)), i)
    png_from_zlib(p, 40, 30, z, idat_split=[None, 7, 100, 1, 50][i],
                  extra=_chunk(b"tEXt", b"k\x00v") if i == 2 else b"")
    paths.append(p)
    streams.append(z)
  Image.fromarray(_depth(rng, 30, 40)).save(str(tmp_path / "pil.png"))
  paths.append(str(tmp_path / "pil.png"))
  raw = bytearray(open(paths[0], "rb").read())
  raw[raw.index(b"IDAT") + 9] ^= 1  # CRC mismatch
  open(str(tmp_path / "crc.png"), "wb").write(bytes(raw))
  Image.fromarray((_depth(rng, 30, 40) % 256).astype(np.uint8)).save(str(tmp_path / "g8.png"))
  write_png16(str(tmp_path / "size.png"), _depth(rng, 31, 40))
  paths += [str(tmp_path / n) for n in ("crc.png", "g8.png", "size.png", "missing.png")]
  buf, need, off, ln, st = depth_gpu.pack(paths, 30, 40, lambda nb: np.zeros(nb, np.uint8))
  sizes = [os.path.getsize(p) if os.path.exists(p) else 0 for p in paths]
  want_off = np.concatenate([[0], np.cumsum([(s + 255) // 256 * 256 for s in sizes])])
  assert list(off) == list(want_off[:-1]) and need == want_off[-1] + 2048
  assert list(st) == [0] * 6 + [2, 1, 3, 4]
  for k in range(5):
    assert bytes(buf[off[k]:off[k] + ln[k]]) == streams[k]
  pil = zlib.decompress(bytes(buf[off[5]:off[5] + ln[5]]))
  assert len(pil) == 30 * 81
  # too small a buffer: nothing read
  with pytest.raises(RuntimeError):
    depth_gpu.pack(paths, 30, 40, lambda nb: np.zeros(nb - 1, np.uint8))


def deflate_matches(z):
  """(output bytes, [(length, distance), ...]) of a zlib stream: a small
  RFC 1951 decoder that records every back-reference (test helper; the
  device decoder's ring / flushed-output split depends on the distances)."""
  pos = [16]  # bit position (after the 2-byte zlib header)
  def bits(n):
    v = 0
    for i in range(n):
      p = pos[0] + i
      v |= ((z[p >> 3] >> (p & 7)) & 1) << i
    pos[0] += n
    return v
  def code(lens):
    cnt = [0] * 16
    for l in lens:
      cnt[l] += 1
    cnt[0] = 0
    nxt, c = [0] * 16, 0
    for L in range(1, 16):
      c = (c + cnt[L - 1]) << 1
      nxt[L] = c
    tab = {}
    for s, l in enumerate(lens):
      if l:
        tab[(l, nxt[l])] = s
        nxt[l] += 1
    return tab
  def sym(tab):
    c = L = 0
    while True:
      c = (c << 1) | bits(1)
      L += 1
      if (L, c) in tab:
        return tab[(L, c)]
  LB = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115,
        131, 163, 195, 227, 258]
  LX = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
  DB = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537,
        2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577]
  DX = [0, 0, 0, 0] + [i // 2 for i in range(2, 28)]
  out, matches = bytearray(), []
  final = 0
  while not final:
    final, typ = bits(1), bits(2)
    if typ == 0:
      pos[0] = (pos[0] + 7) & ~7
      n = bits(16)
      bits(16)
      out += z[pos[0] >> 3:(pos[0] >> 3) + n]
      pos[0] += 8 * n
      continue
    if typ == 1:
      lt = code([8] * 144 + [9] * 112 + [7] * 24 + [8] * 8)
      dt = code([5] * 30)
    else:
      hlit, hdist, hclen = bits(5) + 257, bits(5) + 1, bits(4) + 4
      order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
      cl = [0] * 19
      for i in range(hclen):
        cl[order[i]] = bits(3)
      ct = code(cl)
      lens = []
      while len(lens) < hlit + hdist:
        s = sym(ct)
        if s < 16:
          lens.append(s)
        elif s == 16:
          lens += [lens[-1]] * (3 + bits(2))
        elif s == 17:
          lens += [0] * (3 + bits(3))
        else:
          lens += [0] * (11 + bits(7))
      lt, dt = code(lens[:hlit]), code(lens[hlit:])
    while True:
      s = sym(lt)
      if s < 256:
        out.append(s)
      elif s == 256:
        break
      else:
        n = LB[s - 257] + bits(LX[s - 257])
        ds = sym(dt)
        d = DB[ds] + bits(DX[ds])
        matches.append((n, d))
        for _ in range(n):
          out.append(out[-d])
  return bytes(out), matches


def far_match_stream(rng, period, h, w):
  """Filtered scanlines (filter 0) whose bytes repeat with the given period,
  compressed at level 9: long matches (up to 258 bytes) at distance `period`.
  Returns (zlib stream, raw bytes)."""
  rowb = 2 * w + 1
  base = rng.integers(0, 256, period, dtype=np.uint8)
  raw = np.resize(base, h * rowb)
  raw[::rowb] = 0
  raw = raw.tobytes()
  return zlib.compress(raw, 9), raw


def test_far_match_streams_hold_matches_past_the_ring():
  """The streams of test_gpu_png.py::test_gpu_decode_far_matches: 258-byte
  matches at distances just past the device decoder's 4 KB ring (4096 <
  dist <= 4096 + 257), where a 64-byte copy round would read a slot an
  earlier round of the same copy rewrote; the tracer itself is checked
  against zlib."""
  rng = np.random.default_rng(17)
  for period in (4100, 4166, 4323, 4350):
    z, raw = far_match_stream(rng, period, 24, 720)
    out, matches = deflate_matches(z)
    assert out == raw == zlib.decompress(z)
    far = [m for m in matches if 4096 < m[1] <= 4096 + 257 and m[0] > 64]
    assert len(far) >= 20, (period, len(far))
