"""Per-process runtime of the drop-in API: the default libbopx context and the
cache that keeps model point sets / symmetry sets resident in HBM.

The reference passes `pts` (V x 3) and `syms` (list of dicts) to every
pose_error call (eval_calc_errors.py:315-343); re-uploading them per tuple would
cost more than the kernel, so they are registered once, keyed on the identity
of the caller's arrays (the caller keeps them alive, e.g. models[obj_id]['pts'];
the cache holds a reference so ids are never recycled). Mutating a registered
array in place is not detected — re-create it instead.
"""
import os
import threading

import numpy as np

from . import _lib
from ._lib import _d, _f, _u8, ptr

_tls = threading.local()
_device = int(os.environ.get("BOPX_DEVICE", "0"))


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
    _tls.cache = {}
    _tls.next_id = -1
  return ctx


def resident_object(pts, syms=None, faces=None):
  """obj_id of a transient registered copy of (pts[, syms][, faces])."""
  ctx = context()
  key = (id(pts), id(syms) if syms is not None else None,
         id(faces) if faces is not None else None)
  hit = _tls.cache.get(key)
  if hit is not None:
    return hit[0]
  oid = _tls.next_id
  _tls.next_id -= 1
  ctx.add_object(oid, np.asarray(pts, np.float64), faces)
  if syms is not None:
    from .misc import symmetries_to_array
    s12 = symmetries_to_array(syms)
    if len(s12) == 0:
      raise ValueError("min() arg is an empty sequence")  # what min(es) raises for syms == []
    ctx.set_symmetries(oid, s12)
  _tls.cache[key] = (oid, pts, syms, faces)
  return oid


def pose12(R, t):
  return np.concatenate([np.asarray(R, np.float64).reshape(9),
                         np.asarray(t, np.float64).reshape(3)])


def delta_flags(delta):
  """NumPy >= 2 comparison semantics of `d_diff <= delta` with a float32 d_diff
  (visibility.py:31-37): Python scalars and float32/16 take float32, while
  numpy float64 / >=32-bit integer scalars promote the comparison to float64."""
  if isinstance(delta, (np.floating, np.integer)) and not isinstance(delta, (bool, np.bool_)):
    if isinstance(delta, np.floating):
      return _lib.DELTA_F64 if np.dtype(type(delta)).itemsize >= 8 else 0
    return _lib.DELTA_F64 if np.dtype(type(delta)).itemsize >= 4 else 0
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
