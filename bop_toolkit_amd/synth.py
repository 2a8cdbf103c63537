"""Synthetic BOP-like inputs for tests and benchmarks.

No datasets travel to the GPU box and there is no network, so every benchmark
and parity case is built from seeded synthetic data of the shapes the
reference's BOP datasets have:

* meshes: closed superellipsoid UV grids, V = n_lat * n_lon + 2 vertices,
  F = 2 * n_lat * n_lon triangles ((50, 100) -> 5,002 verts / 10,000 faces,
  the LM-O-like size of BASELINE.json);
* models_info dicts with 'diameter' and optional 'symmetries_discrete' /
  'symmetries_continuous' in the format of models_info.json
  (docs/bop_datasets_format.md; consumed by misc.get_symmetry_transformations,
  misc.py:43-90);
* GT poses uniform on SO(3) at 0.5-1.5 m, estimates perturbed by <= 20 deg and
  N(0, 10 mm), 10 % gross outliers;
* LM-O / YCB-V / T-LESS-like intrinsics (dataset_params.py:345-378).
"""
import numpy as np

LMO_K = np.array([[572.4114, 0.0, 325.2611], [0.0, 573.57043, 242.04899], [0.0, 0.0, 1.0]])
YCBV_K = np.array([[1066.778, 0.0, 312.9869], [0.0, 1067.487, 241.3109], [0.0, 0.0, 1.0]])
TLESS_K = np.array([[1075.65, 0.0, 360.0], [0.0, 1073.90, 270.0], [0.0, 0.0, 1.0]])


def superellipsoid(n_lat, n_lon, axes=(40.0, 30.0, 50.0), eps=0.7, f32=True):
  """Closed UV-grid mesh. Returns (pts V x 3 float64, faces F x 3 uint32).

  With f32=True the coordinates are rounded to float32 values (as
  inout.load_ply reads PLY floats, inout.py:474)."""
  a, b, c = axes

  def f(w, e):
    return np.sign(w) * np.abs(w) ** e

  th = np.pi * np.arange(1, n_lat + 1) / (n_lat + 1)
  ph = 2.0 * np.pi * np.arange(n_lon) / n_lon
  T, P = np.meshgrid(th, ph, indexing="ij")
  x = a * f(np.sin(T), eps) * f(np.cos(P), eps)
  y = b * f(np.sin(T), eps) * f(np.sin(P), eps)
  z = c * f(np.cos(T), eps)
  ring = np.stack([x, y, z], -1).reshape(-1, 3)
  pts = np.concatenate([[[0.0, 0.0, c]], ring, [[0.0, 0.0, -c]]])
  faces = []
  idx = lambda i, j: 1 + i * n_lon + (j % n_lon)
  for j in range(n_lon):  # top fan
    faces.append((0, idx(0, j), idx(0, j + 1)))
  for i in range(n_lat - 1):
    for j in range(n_lon):
      a0, a1, b0, b1 = idx(i, j), idx(i, j + 1), idx(i + 1, j), idx(i + 1, j + 1)
      faces.append((a0, b0, b1))
      faces.append((a0, b1, a1))
  bot = len(pts) - 1
  for j in range(n_lon):  # bottom fan
    faces.append((bot, idx(n_lat - 1, j + 1), idx(n_lat - 1, j)))
  pts = pts.astype(np.float32).astype(np.float64) if f32 else pts
  return pts, np.asarray(faces, np.uint32)


def mesh_diameter(pts, chunk=2048):
  """Exact max pairwise distance (misc.calc_pts_diameter2, misc.py:296-306)."""
  best = 0.0
  for i in range(0, len(pts), chunk):
    d = np.sqrt(((pts[i:i + chunk, None, :] - pts[None, :, :]) ** 2).sum(-1))
    best = max(best, float(d.max()))
  return best


def rot_z(angle):
  c, s = np.cos(angle), np.sin(angle)
  return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])


def models_info_entry(pts, n_disc=1, continuous=False, offset=(0.0, 0.0, 0.0)):
  """models_info.json entry: n_disc-fold discrete z symmetry (n_disc = 1: none),
  optionally a continuous z-axis symmetry."""
  info = {"diameter": mesh_diameter(pts)}
  lo, hi = pts.min(0), pts.max(0)
  info.update({"min_x": lo[0], "min_y": lo[1], "min_z": lo[2],
               "size_x": hi[0] - lo[0], "size_y": hi[1] - lo[1], "size_z": hi[2] - lo[2]})
  if n_disc > 1:
    syms = []
    for j in range(1, n_disc):
      T = np.eye(4)
      T[:3, :3] = rot_z(2.0 * np.pi * j / n_disc)
      syms.append(T.reshape(-1).tolist())
    info["symmetries_discrete"] = syms
  if continuous:
    info["symmetries_continuous"] = [{"axis": [0, 0, 1], "offset": list(offset)}]
  return info


def random_rotations(rng, n):
  q = rng.normal(size=(n, 4))
  q /= np.linalg.norm(q, axis=1, keepdims=True)
  w, x, y, z = q.T
  R = np.stack([
      1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
      2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
      2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)
  return R.reshape(n, 3, 3)


def axis_angle(axis, ang):
  axis = axis / np.linalg.norm(axis, axis=-1, keepdims=True)
  K = np.zeros(axis.shape[:-1] + (3, 3))
  K[..., 0, 1], K[..., 0, 2] = -axis[..., 2], axis[..., 1]
  K[..., 1, 0], K[..., 1, 2] = axis[..., 2], -axis[..., 0]
  K[..., 2, 0], K[..., 2, 1] = -axis[..., 1], axis[..., 0]
  s, c = np.sin(ang)[..., None, None], np.cos(ang)[..., None, None]
  return np.eye(3) + s * K + (1 - c) * (K @ K)


def gt_poses(rng, n, z_range=(500.0, 1500.0), xy=(150.0, 100.0)):
  R = random_rotations(rng, n)
  t = np.stack([rng.uniform(-xy[0], xy[0], n), rng.uniform(-xy[1], xy[1], n),
                rng.uniform(z_range[0], z_range[1], n)], -1)
  return R, t


def perturb(rng, R, t, max_deg=20.0, t_sigma=10.0, outlier_frac=0.1):
  n = len(R)
  ang = np.deg2rad(rng.uniform(0.0, max_deg, n))
  dR = axis_angle(rng.normal(size=(n, 3)), ang)
  Re = dR @ R
  te = t + rng.normal(0.0, t_sigma, size=(n, 3))
  out = rng.random(n) < outlier_frac
  if out.any():
    Re[out] = random_rotations(rng, int(out.sum()))
    te[out] = t[out] + rng.normal(0.0, 100.0, size=(int(out.sum()), 3))
  return Re, te


def pose12(R, t):
  """(n,3,3),(n,3) -> (n,12) [R row-major | t]."""
  R = np.asarray(R, np.float64)
  t = np.asarray(t, np.float64)
  return np.concatenate([R.reshape(R.shape[:-2] + (9,)), t.reshape(t.shape[:-2] + (3,))
                         if t.shape[-1] == 1 else t], -1)
