"""Host-side geometry helpers of the pose-error path (mirror of the hot subset
of bop_toolkit_lib/misc.py).

Symmetry sets, gates and signatures stay on the host (they are O(S) per object
or O(1) per tuple); the per-pixel distance transform runs on the GPU.
"""
import math

import numpy as np

from . import runtime


def rotation_matrix(angle, direction):
  """4x4 rotation about an axis through the origin (transform.py:302-343,
  `point=None` case, which is the only one misc.get_symmetry_transformations
  uses). Same float64 operation order as the reference, so symmetry sets are
  bit-identical."""
  s, c = math.sin(angle), math.cos(angle)
  axis = np.array(direction[:3], dtype=np.float64, copy=True)
  axis /= math.sqrt(np.dot(axis, axis))  # transform.unit_vector, transform.py:1751-1753
  R = np.diag([c, c, c])
  R += np.outer(axis, axis) * (1.0 - c)
  axis *= s
  R += np.array([[0.0, -axis[2], axis[1]],
                 [axis[2], 0.0, -axis[0]],
                 [-axis[1], axis[0], 0.0]])
  M = np.identity(4)
  M[:3, :3] = R
  return M


def get_symmetry_transformations(model_info, max_sym_disc_step):
  """Symmetry transformations of an object (misc.py:43-90).

  Returns a list of {'R': 3x3, 't': 3x1}. As in the reference, the identity
  is part of the set only when the object has no continuous symmetry: with a
  continuous axis the set is {cont_i o disc_j}, i = 1..n-1 (misc.py:74,80-88).
  """
  discrete = [{"R": np.eye(3), "t": np.array([[0, 0, 0]]).T}]
  for sym in model_info.get("symmetries_discrete", []):
    T = np.reshape(sym, (4, 4))
    discrete.append({"R": T[:3, :3], "t": T[:3, 3].reshape((3, 1))})

  continuous = []
  for sym in model_info.get("symmetries_continuous", []):
    axis = np.array(sym["axis"])
    offset = np.array(sym["offset"]).reshape((3, 1))
    steps = int(np.ceil(np.pi / max_sym_disc_step))
    step = 2.0 * np.pi / steps
    for i in range(1, steps):
      R = rotation_matrix(i * step, axis)[:3, :3]
      continuous.append({"R": R, "t": -R.dot(offset) + offset})

  if not continuous:
    return list(discrete)
  out = []
  for d in discrete:
    for cs in continuous:
      out.append({"R": cs["R"].dot(d["R"]), "t": cs["R"].dot(d["t"]) + cs["t"]})
  return out


def symmetries_to_array(syms):
  """List of {'R','t'} -> S x 12 float64 rows [R row-major | t] (the layout
  uploaded by bopx_set_symmetries)."""
  if len(syms) == 0:
    return np.zeros((0, 12))
  R = np.stack([np.asarray(s["R"], np.float64).reshape(9) for s in syms])
  t = np.stack([np.asarray(s["t"], np.float64).reshape(3) for s in syms])
  return np.ascontiguousarray(np.concatenate([R, t], 1))


def transform_pts_Rt(pts, R, t):
  """(R pts^T + t)^T (misc.py:266-276)."""
  assert pts.shape[1] == 3
  return (R.dot(pts.T) + t.reshape((3, 1))).T


def project_pts(pts, K, R, t):
  """Pinhole projection of 3D points (misc.py:93-107)."""
  assert pts.shape[1] == 3
  P = K.dot(np.hstack((R, t)))
  pts_h = np.hstack((pts, np.ones((pts.shape[0], 1))))
  pts_im = P.dot(pts_h.T)
  pts_im /= pts_im[2, :]
  return pts_im[:2, :].T


def depth_im_to_dist_im_fast(depth_im, K):
  """Depth image -> distance-from-camera image (misc.py:143-163), on the GPU.

  float64 result with the reference's exact operation order:
  sqrt((pX*d)**2 + (pY*d)**2 + d**2), pX = (x - cx) / fx, pY = (y - cy) / fy.
  (The reference's Precomputer cache, misc.py:110-140, is not reproduced: it
  returns stale coefficients when the frame size changes with the same K.)"""
  return runtime.dist_im(depth_im, K)


def depth_im_to_dist_im(depth_im, K):
  """Same as depth_im_to_dist_im_fast (misc.py:166-189 is the slow variant)."""
  return runtime.dist_im(depth_im, K)


def overlapping_sphere_projections(radius, p1, p2):
  """Approximate overlap test of two projected spheres (misc.py:309-331)."""
  if p1[2] == 0 or p2[2] == 0:
    return False
  proj1 = (p1 / p1[2])[:2]
  proj2 = (p2 / p2[2])[:2]
  proj_dist = np.linalg.norm(proj1 - proj2)
  proj_dist_thresh = radius * (1.0 / p1[2] + 1.0 / p2[2])
  return proj_dist < proj_dist_thresh


def get_error_signature(error_type, n_top, **kwargs):
  """Directory signature of an error set (misc.py:334-350)."""
  sig = "error=" + error_type + "_ntop=" + str(n_top)
  if error_type == "vsd":
    tau = kwargs["vsd_tau"]
    tau_str = "inf" if tau == float("inf") else "{:.3f}".format(tau)
    sig += "_delta={:.3f}_tau={}".format(kwargs["vsd_delta"], tau_str)
  return sig


def calc_pts_diameter(pts):
  """Max pairwise distance of a point set (misc.py:279-306)."""
  pts = np.asarray(pts, np.float64)
  best = -1.0  # the reference's value for an empty set
  # rows per chunk: ~4M pairwise entries (~100 MB of float64 temporaries)
  chunk = max(1, 2 ** 22 // max(len(pts), 1))
  for i in range(0, len(pts), chunk):
    d = ((pts[i:i + chunk, None, :] - pts[None, :, :]) ** 2).sum(-1)
    best = max(best, float(np.sqrt(d.max())))
  return best


def log(s):
  """Timestamped progress line, flushed (misc.py:18-33)."""
  import datetime
  import sys
  now = datetime.datetime.now(datetime.timezone.utc)
  sys.stdout.write("{}/{}|{:02d}:{:02d}:{:02d}: {}\n".format(
      now.month, now.day, now.hour, now.minute, now.second, s))
  sys.stdout.flush()


def get_score_signature(correct_th, visib_gt_min):
  """Signature of a score setting (misc.py:353-361)."""
  return "th=" + "-".join("{:.3f}".format(t) for t in correct_th) + \
      "_min-visib={:.3f}".format(visib_gt_min)


def calc_pts_diameter2(pts):
  """Same value as calc_pts_diameter (misc.py:296-306 is the all-pairs variant;
  like its np.max over an empty cdist, an empty set raises ValueError)."""
  if len(pts) == 0:
    raise ValueError("zero-size array to reduction operation maximum which has no identity")
  return calc_pts_diameter(pts)


def ensure_dir(path):
  """Create a directory (and parents) if missing (misc.py:34-40)."""
  import os
  if not os.path.exists(path):
    os.makedirs(path)


def clip_pt_to_im(pt, im_size):
  """Clip a 2D point to the image frame (misc.py:191-199)."""
  return [min(max(pt[0], 0), im_size[0] - 1), min(max(pt[1], 0), im_size[1] - 1)]


def calc_3d_bbox(xs, ys, zs):
  """(x, y, z, w, h, d) of a 3D point set (misc.py:221-233)."""
  lo = [xs.min(), ys.min(), zs.min()]
  hi = [xs.max(), ys.max(), zs.max()]
  return [lo[0], lo[1], lo[2], hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]]


def calc_2d_bbox(xs, ys, im_size=None, clip=False):
  """(x, y, w, h) of a point set, w = max - min (misc.py:202-218)."""
  lo = [xs.min(), ys.min()]
  hi = [xs.max(), ys.max()]
  if clip:
    assert im_size is not None
    lo = clip_pt_to_im(lo, im_size)
    hi = clip_pt_to_im(hi, im_size)
  return [lo[0], lo[1], hi[0] - lo[0], hi[1] - lo[1]]


def iou(bb_a, bb_b):
  """Intersection over union of two (x, y, w, h) boxes (misc.py:236-263)."""
  ax1, ay1 = bb_a[0] + bb_a[2], bb_a[1] + bb_a[3]
  bx1, by1 = bb_b[0] + bb_b[2], bb_b[1] + bb_b[3]
  w = min(ax1, bx1) - max(bb_a[0], bb_b[0])
  h = min(ay1, by1) - max(bb_a[1], bb_b[1])
  if w > 0 and h > 0:
    inter = w * h
    return inter / float(bb_a[2] * bb_a[3] + bb_b[2] * bb_b[3] - inter)
  return 0.0
