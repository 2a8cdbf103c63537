"""Pose-error functions with the signatures of bop_toolkit_lib/pose_error.py,
evaluated by the gfx950 kernels of libbopx.

Drop-in: `from bop_toolkit_amd import pose_error` in place of
`from bop_toolkit_lib import pose_error` (scripts/eval_calc_errors.py:16).
Every per-tuple function below is a batch of one through the C-ABI; batched
throughput comes from bop_toolkit_amd.batch (one launch per batch).

Return values are Python/NumPy float64 like the reference. VSD results are
bit-identical to the reference given the same depth maps; MSSD/MSPD/ADD/ADI/
PROJ agree to float64 rounding (<< 1e-4 mm / px).
"""
import math

import numpy as np

from . import _lib
from . import misc
from . import runtime
from ._lib import _d, _f, _i32, ptr
from .renderer_hip import RendererHIP


def _cost_code(cost_type):
  return {"step": _lib.COST_STEP, "tlinear": _lib.COST_TLINEAR}.get(cost_type)


def _tau_chunks(n):
  """[k0, k1) ranges of at most MAX_TAUS thresholds (one kernel call each; the
  reference takes any number of taus)."""
  return [(k0, min(k0 + _lib.MAX_TAUS, n)) for k0 in range(0, n, _lib.MAX_TAUS)]


# Per-call constants of the fused VSD path (inputs the library only reads): the
# one-tuple frame index, obj_id arrays and tau chunks, with their ctypes
# pointers made once (numpy's .ctypes costs ~4 us per array and call).
_ZERO_I32 = np.zeros(1, np.int32)
_ZERO_I32_P = ptr(_ZERO_I32, _i32)
_CONST_CACHE = {}


def _const(key, make, ct):
  hit = _CONST_CACHE.get(key)
  if hit is None:
    if len(_CONST_CACHE) > 256:
      _CONST_CACHE.clear()
    arr = make()
    hit = _CONST_CACHE[key] = (arr, ptr(arr, ct))
  return hit[1]


def vsd(R_est, t_est, R_gt, t_gt, depth_test, K, delta, taus, normalized_by_diameter,
        diameter, renderer, obj_id, cost_type="step"):
  """Visible Surface Discrepancy (pose_error.py:17-93).

  With a RendererHIP the two renders, three distance images, both visibility
  masks and the per-tau costs run in one fused kernel (k_vsd). With any other
  duck-typed renderer (renderer.render_object(...)['depth']), its depth maps
  are evaluated on the GPU (k_vsd_depths).
  Returns a list of len(taus) numpy.float64 errors (pose_error.py:90-91), or
  the Python floats [1.0] * len(taus) for an empty visibility union
  (pose_error.py:75-76); the kernels report the union count for that choice.
  """
  taus = [float(t) for t in taus]
  ctx = runtime.context()
  fx, fy, cx, cy = float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2])
  depth_test = np.ascontiguousarray(depth_test, np.float32)
  H, W = depth_test.shape
  flags = runtime.delta_flags(delta) | _lib.VSD_UNIONS
  tau_arr = np.asarray(taus, np.float64)
  out = np.empty(len(taus) + 1, np.float64)  # errors, then the union count
  code = _cost_code(cost_type)
  if isinstance(renderer, RendererHIP) and renderer.ctx is ctx and code is not None and taus:
    oid = int(obj_id)
    p_ids = _const(("id", oid), lambda: np.array([oid], np.int32), _i32)
    # pose_est | pose_gt | cam | diameter | results | union in one float64 block
    # (a tau chunk writes its union count after its results: into the next
    # chunk's first slot, which that chunk then overwrites, or the last slot)
    nt = len(taus)
    blk = np.empty(30 + nt, np.float64)
    blk[0:9] = np.asarray(R_est, np.float64).reshape(9)
    blk[9:12] = np.asarray(t_est, np.float64).reshape(3)
    blk[12:21] = np.asarray(R_gt, np.float64).reshape(9)
    blk[21:24] = np.asarray(t_gt, np.float64).reshape(3)
    blk[24:28] = (fx, fy, cx, cy)
    blk[28] = float(diameter)
    base = blk.ctypes.data
    step = blk.itemsize
    p_pe, p_pg = _lib.cast_ptr(base, _d), _lib.cast_ptr(base + 12 * step, _d)
    p_cam, p_dia = _lib.cast_ptr(base + 24 * step, _d), _lib.cast_ptr(base + 28 * step, _d)
    p_dep = ptr(depth_test, _f)
    for k0, k1 in _tau_chunks(nt):  # the kernels take MAX_TAUS per call
      key = ("taus", tau_arr[k0:k1].tobytes())  # bit-exact (signed zeros, NaNs)
      p_tau = _const(key, lambda: np.ascontiguousarray(tau_arr[k0:k1]), _d)
      ctx.call("bopx_vsd_batch", 1, p_ids, p_pe, p_pg, _ZERO_I32_P, p_dep, 1, W, H, p_cam,
               float(delta), flags, p_tau, k1 - k0, int(bool(normalized_by_diameter)), p_dia,
               code, _lib.cast_ptr(base + (29 + k0) * step, _d))
    return _vsd_result(blk[29:29 + nt], blk[29 + nt])
  depth_est = renderer.render_object(obj_id, R_est, t_est, fx, fy, cx, cy)["depth"]
  depth_gt = renderer.render_object(obj_id, R_gt, t_gt, fx, fy, cx, cy)["depth"]
  de = np.ascontiguousarray(depth_est, np.float32)
  dg = np.ascontiguousarray(depth_gt, np.float32)
  if not taus:
    return []
  for k0, k1 in _tau_chunks(len(taus)):
    part, o = np.ascontiguousarray(tau_arr[k0:k1]), np.empty(k1 - k0 + 1, np.float64)
    ctx.call("bopx_vsd_from_depths", W, H, ptr(depth_test, _f), ptr(de, _f), ptr(dg, _f), fx,
             fy, cx, cy, float(delta), flags, ptr(part, _d), k1 - k0,
             int(bool(normalized_by_diameter)), float(diameter),
             code if code is not None else 99, ptr(o, _d))
    out[k0:k1] = o[:-1]
    out[-1] = o[-1]
  return _vsd_result(out[:-1], out[-1])


def _vsd_result(errors, union):
  """The reference's return value: numpy.float64 elements (pose_error.py:90-91,
  `(np.sum(costs) + comp) / float(union)`), Python floats for an empty union
  (:75-76)."""
  if union == 0:
    return [1.0] * len(errors)
  return list(np.array(errors, np.float64))


def _point_error(name, R_est, t_est, R_gt, t_gt, pts, syms=None, K=None):
  ctx = runtime.context()
  oid = runtime.resident_object(pts, syms)
  p_ids = _const(("id", oid), lambda: np.array([oid], np.int32), _i32)
  # pose_est | pose_gt | K | result in one float64 block (see vsd)
  blk = np.empty(34, np.float64)
  blk[0:9] = np.asarray(R_est, np.float64).reshape(9)
  blk[9:12] = np.asarray(t_est, np.float64).reshape(3)
  blk[12:21] = np.asarray(R_gt, np.float64).reshape(9)
  blk[21:24] = np.asarray(t_gt, np.float64).reshape(3)
  base, step = blk.ctypes.data, blk.itemsize
  p_pe, p_pg = _lib.cast_ptr(base, _d), _lib.cast_ptr(base + 12 * step, _d)
  p_out = _lib.cast_ptr(base + 33 * step, _d)
  if K is not None:
    blk[24:33] = np.asarray(K, np.float64).reshape(9)
    ctx.call(name, 1, p_ids, p_pe, p_pg, _lib.cast_ptr(base + 24 * step, _d), p_out)
  else:
    ctx.call(name, 1, p_ids, p_pe, p_pg, p_out)
  return np.float64(blk[33])


def mssd(R_est, t_est, R_gt, t_gt, pts, syms):
  """Maximum Symmetry-Aware Surface Distance (pose_error.py:96-118)."""
  return _point_error("bopx_mssd_batch", R_est, t_est, R_gt, t_gt, pts, syms)


def mspd(R_est, t_est, R_gt, t_gt, K, pts, syms):
  """Maximum Symmetry-Aware Projection Distance (pose_error.py:121-144)."""
  return _point_error("bopx_mspd_batch", R_est, t_est, R_gt, t_gt, pts, syms, K=K)


def add(R_est, t_est, R_gt, t_gt, pts):
  """Average Distance of model points, ADD (pose_error.py:147-161)."""
  return _point_error("bopx_add_batch", R_est, t_est, R_gt, t_gt, pts)


def adi(R_est, t_est, R_gt, t_gt, pts):
  """ADD for indistinguishable views, ADI (pose_error.py:164-184): mean
  distance from each GT-pose vertex to its exact nearest estimated-pose vertex
  (brute force on the GPU instead of scipy's cKDTree; same NN distances)."""
  return _point_error("bopx_adi_batch", R_est, t_est, R_gt, t_gt, pts)


def proj(R_est, t_est, R_gt, t_gt, K, pts):
  """Mean 2D projection distance (pose_error.py:217-232)."""
  return _point_error("bopx_proj_batch", R_est, t_est, R_gt, t_gt, pts, K=K)


def re(R_est, R_gt):
  """Rotational error in degrees (pose_error.py:187-202). O(1) host math."""
  assert R_est.shape == R_gt.shape == (3, 3)
  cos = float(0.5 * (np.trace(R_est.dot(np.linalg.inv(R_gt))) - 1.0))
  cos = min(1.0, max(-1.0, cos))
  return 180.0 * math.acos(cos) / np.pi


def te(t_est, t_gt):
  """Translational error (pose_error.py:205-214). O(1) host math."""
  assert t_est.size == t_gt.size == 3
  return np.linalg.norm(t_gt - t_est)


def _cover(R_est, t_est, R_gt, t_gt, K, renderer, obj_id):
  """[union, inter, est bbox x0 y0 x1 y1, gt bbox x0 y0 x1 y1] of the two
  rendered silhouettes (depth > 0). RendererHIP: both renders fused into one
  k_vsd launch in silhouette mode; other renderers: their depth maps are
  compared on the GPU (k_cover_depths)."""
  ctx = runtime.context()
  fx, fy, cx, cy = float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2])
  out = np.empty(10, np.float64)
  if isinstance(renderer, RendererHIP) and renderer.ctx is ctx:
    ids = np.array([obj_id], np.int32)
    pe, pg = runtime.pose12(R_est, t_est), runtime.pose12(R_gt, t_gt)
    fi = np.zeros(1, np.int32)
    cam = np.array([fx, fy, cx, cy], np.float64)
    ctx.call("bopx_cover_batch", 1, ptr(ids, _i32), ptr(pe, _d), ptr(pg, _d), ptr(fi, _i32), 1,
             renderer.width, renderer.height, ptr(cam, _d), ptr(out, _d))
  else:
    de = np.ascontiguousarray(renderer.render_object(obj_id, R_est, t_est, fx, fy, cx, cy)
                              ["depth"], np.float32)
    dg = np.ascontiguousarray(renderer.render_object(obj_id, R_gt, t_gt, fx, fy, cx, cy)
                              ["depth"], np.float32)
    assert de.shape == dg.shape
    ctx.call("bopx_cover_from_depths", de.shape[1], de.shape[0], ptr(de, _f), ptr(dg, _f),
             ptr(out, _d))
  return out


def cus_from_cover(cov):
  """1 - |inter| / |union| of two masks, 1.0 for an empty union."""
  union, inter = float(cov[0]), float(cov[1])
  return 1.0 - inter / union if union > 0 else 1.0


def bbox_from_cover(cov, k):
  """misc.calc_2d_bbox of mask k (0 = est, 1 = gt) from a cover row."""
  x0, y0, x1, y1 = (int(v) for v in cov[2 + 4 * k:6 + 4 * k])
  if x1 < 0:  # numpy's error for xs.min() of an empty mask
    raise ValueError("zero-size array to reduction operation minimum which has no identity")
  return [x0, y0, x1 - x0, y1 - y0]


def cus(R_est, t_est, R_gt, t_gt, K, renderer, obj_id):
  """Complement over Union of the projected silhouettes (pose_error.py:256-286)."""
  return np.float64(cus_from_cover(_cover(R_est, t_est, R_gt, t_gt, K, renderer, obj_id)))


def cou_bb_proj(R_est, t_est, R_gt, t_gt, K, renderer, obj_id):
  """Complement over Union of the silhouettes' 2D bounding boxes (pose_error.py:300-330)."""
  cov = _cover(R_est, t_est, R_gt, t_gt, K, renderer, obj_id)
  return 1.0 - misc.iou(bbox_from_cover(cov, 0), bbox_from_cover(cov, 1))


def cou_mask(mask_est, mask_gt):
  """Complement over Union of two given binary masks (pose_error.py:233-253).
  Host bookkeeping on caller-provided masks."""
  me, mg = np.asarray(mask_est).astype(bool), np.asarray(mask_gt).astype(bool)
  union = float(np.logical_or(me, mg).sum())
  return 1.0 - np.logical_and(me, mg).sum() / union if union > 0 else 1.0


def cou_bb(bb_est, bb_gt):
  """Complement over Union of two 2D boxes (x, y, w, h) (pose_error.py:289-297)."""
  return 1.0 - misc.iou(bb_est, bb_gt)
