"""Per-process runtime of the drop-in API: the default libbopx context and the
cache that keeps model point sets / symmetry sets resident in HBM.

The reference passes `pts` (V x 3) and `syms` (list of dicts) to every
pose_error call (eval_calc_errors.py:315-343); re-uploading them per tuple would
cost more than the kernel, so they are registered once and reused:

* objects are keyed on their CONTENT (shape, dtype and a BLAKE2b digest of the
  bytes of pts / syms / faces), so equal point sets share one HBM slot even when
  the caller builds a fresh array per call (`model['pts'] * 1.0`);
* a small identity map in front of it (the caller's array objects -> content
  key) skips the digest when the same arrays come back; it holds references to
  those arrays so their ids are never recycled while mapped;
* both maps are LRU-bounded: evicting an object calls remove_object, which
  frees its HBM slot. Mutating an array in place after a call is not detected
  by the identity map — re-create it instead.
"""
import collections
import hashlib
import os
import threading

import numpy as np

from . import _lib
from ._lib import _d, _f, _u8, ptr

_tls = threading.local()
_device = int(os.environ.get("BOPX_DEVICE", "0"))
# LRU bounds of the drop-in object cache (resident objects; identity entries).
MAX_RESIDENT = int(os.environ.get("BOPX_MAX_RESIDENT", "64"))
MAX_IDENTITY = 4 * MAX_RESIDENT


def set_device(device):
  """Select the HIP device used by contexts created afterwards in this thread."""
  global _device
  _device = int(device)
  _tls.ctx = None


def context():
  ctx = getattr(_tls, "ctx", None)
  if ctx is None:
    ctx = _lib.Context(_device)
    _tls.ctx = ctx
    _tls.by_id = collections.OrderedDict()       # identity key -> (content key, arrays)
    _tls.by_content = collections.OrderedDict()  # content key -> obj_id
    _tls.next_id = -1
  return ctx


def _digest(a):
  if a is None:
    return None
  a = np.ascontiguousarray(a)
  return (a.shape, a.dtype.str, hashlib.blake2b(a.view(np.uint8).reshape(-1),
                                                digest_size=16).digest())


def resident_count():
  """Number of objects the drop-in cache currently keeps in HBM (this thread)."""
  context()
  return len(_tls.by_content)


def resident_object(pts, syms=None, faces=None):
  """obj_id of a transient registered copy of (pts[, syms][, faces])."""
  ctx = context()
  ikey = (id(pts), id(syms) if syms is not None else None,
          id(faces) if faces is not None else None)
  hit = _tls.by_id.get(ikey)
  if hit is not None and hit[0] in _tls.by_content:
    _tls.by_id.move_to_end(ikey)
    _tls.by_content.move_to_end(hit[0])
    return _tls.by_content[hit[0]]
  pts64 = np.ascontiguousarray(pts, np.float64)
  s12 = None
  if syms is not None:
    from .misc import symmetries_to_array
    s12 = symmetries_to_array(syms)
    if len(s12) == 0:
      raise ValueError("min() arg is an empty sequence")  # what min(es) raises for syms == []
  f32 = None if faces is None else np.ascontiguousarray(faces, np.uint32)
  ckey = (_digest(pts64), _digest(s12), _digest(f32))
  oid = _tls.by_content.get(ckey)
  if oid is None:
    oid = _tls.next_id
    _tls.next_id -= 1
    ctx.add_object(oid, pts64, f32)
    if s12 is not None:
      ctx.set_symmetries(oid, s12)
    _tls.by_content[ckey] = oid
    while len(_tls.by_content) > MAX_RESIDENT:
      old_key, old_oid = _tls.by_content.popitem(last=False)
      ctx.remove_object(old_oid)
      for k in [k for k, v in _tls.by_id.items() if v[0] == old_key]:
        del _tls.by_id[k]
  else:
    _tls.by_content.move_to_end(ckey)
  _tls.by_id[ikey] = (ckey, pts, syms, faces)
  _tls.by_id.move_to_end(ikey)
  while len(_tls.by_id) > MAX_IDENTITY:
    _tls.by_id.popitem(last=False)
  return oid


def pose12(R, t):
  return np.concatenate([np.asarray(R, np.float64).reshape(9),
                         np.asarray(t, np.float64).reshape(3)])


def delta_flags(delta):
  """Comparison semantics of `d_diff <= delta` for a float32 d_diff
  (visibility.py:31-37) under the reference's own runtime.

  The reference only runs on NumPy < 1.24 (it uses the removed aliases
  np.float / np.bool, inout.py:153, pose_error.py:63), whose legacy value-based
  casting compares a float32 array with ANY scalar delta (Python float, numpy
  float64 or integer) in float32 — unless the value does not fit in float32
  (|delta| > FLT_MAX), which promotes the comparison to float64. That is the
  semantics followed here for every scalar type. (NumPy >= 2 would promote a
  numpy float64 scalar to a float64 comparison; eval_calc_errors passes Python
  floats, for which both agree.)"""
  d = float(delta)
  if d == d and abs(d) != float("inf") and abs(d) > float(np.finfo(np.float32).max):
    return _lib.DELTA_F64
  return 0


def dist_im(depth_im, K):
  ctx = context()
  d = np.ascontiguousarray(depth_im, np.float32)
  if d.ndim != 2:
    raise ValueError("depth_im must be 2-D")
  H, W = d.shape
  out = np.empty((H, W), np.float64)
  ctx.call("bopx_dist_im", W, H, ptr(d, _f), float(K[0, 0]), float(K[1, 1]), float(K[0, 2]),
           float(K[1, 2]), ptr(out, _d))
  return out


def visib_mask(d_test, d_model, delta, visib_mode, visib_gt=None):
  ctx = context()
  mode = {"bop18": _lib.VISIB_BOP18, "bop19": _lib.VISIB_BOP19}.get(visib_mode)
  if mode is None:
    raise ValueError("Unknown visibility mode.")
  t = np.ascontiguousarray(d_test, np.float64)
  m = np.ascontiguousarray(d_model, np.float64)
  vg = None if visib_gt is None else np.ascontiguousarray(np.asarray(visib_gt) != 0, np.uint8)
  out = np.empty(t.shape, np.uint8)
  ctx.call("bopx_visib_mask", t.size, ptr(t, _d), ptr(m, _d), ptr(vg, _u8), float(delta),
           delta_flags(delta), mode, ptr(out, _u8))
  return out.view(bool)
