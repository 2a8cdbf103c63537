"""CPU model of occlusion culling for k_vsd (design study, not product code).

For the bench workload (superellipsoid objects, YCB-V K, 640x480) it counts the
(pose, meshlet, tile) entries of k_vsd and how many of them an entry-level
occlusion test could skip: an entry is skippable when every pixel of its
rectangle inside the tile already holds q = 1/Z >= the meshlet's largest
possible q (1 / the nearest OBB corner Z) in the FINAL q-buffer of that pose
(the upper bound of any front-to-back order). Meshlets follow runtime.cpp
(Hilbert order of face centroids, greedy <= 64 triangles / <= 64 vertices, OBB
from the vertex covariance).

  python tools/cull_model.py --tuples 60
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bop_toolkit_amd import synth  # noqa: E402
from oracle import oracle  # noqa: E402


def hilbert3(q):
  x = [int(q[0]), int(q[1]), int(q[2])]
  Q = 1 << 9
  while Q > 1:
    P = Q - 1
    for i in range(3):
      if x[i] & Q:
        x[0] ^= P
      else:
        t = (x[0] ^ x[i]) & P
        x[0] ^= t
        x[i] ^= t
    Q >>= 1
  for i in range(1, 3):
    x[i] ^= x[i - 1]
  t = 0
  Q = 1 << 9
  while Q > 1:
    if x[2] & Q:
      t ^= Q - 1
    Q >>= 1
  for i in range(3):
    x[i] ^= t
  key = 0
  for b in range(9, -1, -1):
    for i in range(3):
      key = (key << 1) | ((x[i] >> b) & 1)
  return key


def meshlets(pts, faces):
  v = pts.astype(np.float32)
  lo, hi = v.min(0), v.max(0)
  cen = v[faces].sum(1) / np.float32(3)
  u = np.where(hi > lo, (cen - lo) / np.where(hi > lo, hi - lo, 1), 0)
  q = np.clip(u * 1023, 0, 1023).astype(np.uint32)
  keys = np.array([hilbert3(r) for r in q])
  order = np.argsort(keys, kind="stable")
  out = []
  f = 0
  while f < len(order):
    used, tris = set(), []
    while f < len(order) and len(tris) < 64:
      t = faces[order[f]]
      fresh = [x for x in t if x not in used]
      if len(used) + len(fresh) > 64:
        break
      used.update(t.tolist())
      tris.append(order[f])
      f += 1
    ids = np.array(sorted(used))
    P = v[ids].astype(np.float64)
    mean = P.mean(0)
    w, ax = np.linalg.eigh(np.cov((P - mean).T) if len(P) > 1 else np.eye(3))
    t = (P - mean) @ ax
    lo3, hi3 = t.min(0), t.max(0)
    pad = 1e-4 * (hi3 - lo3).max() + 1e-3
    lo3, hi3 = lo3 - pad, hi3 + pad
    corners = np.array([[(hi3 if c & (1 << k) else lo3)[k] for k in range(3)] for c in range(8)])
    out.append({"tris": np.array(tris), "corners": mean + corners @ ax.T})
  return out


def rect_of(corners, R, t, K, W, H):
  X = corners @ R.T + t
  if (X[:, 2] <= 0).any():
    return (0, 0, W - 1, H - 1), np.inf
  u = K[0, 0] * X[:, 0] / X[:, 2] + K[0, 2]
  v = K[1, 1] * X[:, 1] / X[:, 2] + K[1, 2]
  x0, x1 = np.ceil(u.min() - 0.5 - 0.0625), np.floor(u.max() - 0.5 + 0.0625)
  y0, y1 = np.ceil(v.min() - 0.5 - 0.0625), np.floor(v.max() - 0.5 + 0.0625)
  if x1 < 0 or y1 < 0 or x0 > W - 1 or y0 > H - 1:
    return None, 0.0
  return (int(max(x0, 0)), int(max(y0, 0)), int(min(x1, W - 1)), int(min(y1, H - 1))), \
      1.0 / X[:, 2].min()


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--tuples", type=int, default=40)
  ap.add_argument("--objects", type=int, default=6)
  ap.add_argument("--tile", type=int, default=64)
  ap.add_argument("--margin", type=float, default=2.0 ** -8)
  a = ap.parse_args()
  rng = np.random.default_rng(0)
  W, H, K, T = 640, 480, synth.YCBV_K, a.tile
  objs = []
  for _ in range(a.objects):
    pts, faces = synth.superellipsoid(50, 100, tuple(rng.uniform(30, 100, 3)),
                                      float(rng.uniform(0.5, 1.0)))
    objs.append((pts, faces, meshlets(pts, faces)))
  Rg, tg = synth.gt_poses(rng, a.tuples)
  Re, te = synth.perturb(rng, Rg, tg)
  n_ent = n_cull = n_tri = n_tri_cull = 0
  for i in range(a.tuples):
    pts, faces, ml = objs[i % a.objects]
    poses = [(Re[i], te[i]), (Rg[i], tg[i])]
    rects, Q = [], []
    for R, t in poses:
      d = oracle.render_depth(pts, faces, R, t, K[0, 0], K[1, 1], K[0, 2], K[1, 2], W, H)
      Q.append(np.where(d > 0, 1.0 / np.where(d > 0, d, 1), 0.0))
      rects.append([rect_of(m["corners"], R, t, K, W, H) for m in ml])
    rr = [r for rs in rects for r, _ in rs if r is not None]
    if not rr:
      continue
    rx0, ry0 = min(r[0] for r in rr), min(r[1] for r in rr)
    rx1, ry1 = max(r[2] for r in rr), max(r[3] for r in rr)
    for ty in range(ry0, ry1 + 1, T):
      for tx in range(rx0, rx1 + 1, T):
        tx1, ty1 = min(tx + T - 1, rx1), min(ty + T - 1, ry1)
        for p in range(2):
          for m, (r, qmax) in zip(ml, rects[p]):
            if r is None or r[0] > tx1 or r[2] < tx or r[1] > ty1 or r[3] < ty:
              continue
            n_ent += 1
            n_tri += len(m["tris"])
            x0, y0, x1, y1 = max(r[0], tx), max(r[1], ty), min(r[2], tx1), min(r[3], ty1)
            if Q[p][y0:y1 + 1, x0:x1 + 1].min() >= qmax * (1 + a.margin):
              n_cull += 1
              n_tri_cull += len(m["tris"])
  print("entries %d (%.1f per tuple), cullable %.1f %%, triangle-weighted %.1f %%" %
        (n_ent, n_ent / a.tuples, 100.0 * n_cull / max(n_ent, 1),
         100.0 * n_tri_cull / max(n_tri, 1)))


if __name__ == "__main__":
  main()


def simulate(tuples=10, lag=16, T=64, margin=2.0 ** -8, seed=0):
  """Queue-order simulation: entry k of a tile's queue is tested against the
  q-buffer holding the entries 0..k-lag-1 (lag = entries in flight). Orders:
  'index' (meshlet order), 'near' (nearest OBB corner first), 'lpt' (overlap
  >= 1024 px first, as k_vsd)."""
  rng = np.random.default_rng(seed)
  W, H, K = 640, 480, synth.YCBV_K
  pts, faces = synth.superellipsoid(50, 100, tuple(rng.uniform(30, 100, 3)),
                                    float(rng.uniform(0.5, 1.0)))
  ml = meshlets(pts, faces)
  Rg, tg = synth.gt_poses(rng, tuples)
  Re, te = synth.perturb(rng, Rg, tg)
  res = {k: [0, 0] for k in ("index", "near", "lpt", "ideal", "b2", "b4", "b8")}
  for i in range(tuples):
    poses = [(Re[i], te[i]), (Rg[i], tg[i])]
    per = []  # per pose: list of (rect, qmax, Qm) per meshlet
    for R, t in poses:
      lst = []
      for m in ml:
        r, qmax = rect_of(m["corners"], R, t, K, W, H)
        if r is None:
          lst.append(None)
          continue
        d = oracle.render_depth(pts, faces[m["tris"]], R, t, K[0, 0], K[1, 1], K[0, 2], K[1, 2],
                                W, H)
        lst.append((r, qmax, np.where(d > 0, 1.0 / np.where(d > 0, d, 1), 0.0)))
      per.append(lst)
    rr = [e[0] for lst in per for e in lst if e is not None]
    rx0, ry0 = min(r[0] for r in rr), min(r[1] for r in rr)
    rx1, ry1 = max(r[2] for r in rr), max(r[3] for r in rr)
    for ty in range(ry0, ry1 + 1, T):
      for tx in range(rx0, rx1 + 1, T):
        tx1, ty1 = min(tx + T - 1, rx1), min(ty + T - 1, ry1)
        ents = []
        for p in range(2):
          for e in per[p]:
            if e is None:
              continue
            r = e[0]
            if r[0] > tx1 or r[2] < tx or r[1] > ty1 or r[3] < ty:
              continue
            x0, y0, x1, y1 = max(r[0], tx), max(r[1], ty), min(r[2], tx1), min(r[3], ty1)
            ents.append((p, e, (x0, y0, x1, y1), (x1 - x0 + 1) * (y1 - y0 + 1)))
        final = [np.zeros((H, W)), np.zeros((H, W))]
        for p, e, _, _ in ents:
          final[p] = np.maximum(final[p], e[2])
        orders = {
            "index": list(range(len(ents))),
            "near": sorted(range(len(ents)), key=lambda k: -ents[k][1][1]),
            "lpt": [k for k in range(len(ents)) if ents[k][3] >= 1024] +
                   [k for k in range(len(ents)) if ents[k][3] < 1024][::-1],
        }
        if not ents:
          continue
        qs = np.array([ents[k][1][1] for k in range(len(ents))])
        for nb in (2, 4, 8):  # buckets of the tile's qmax range, nearest first
          lo, hi = qs.min(), qs.max()
          b = np.minimum(((hi - qs) / max(hi - lo, 1e-30) * nb).astype(int), nb - 1)
          orders["b%d" % nb] = [k for bb in range(nb) for k in range(len(ents)) if b[k] == bb]
        for name, order in orders.items():
          cur = [np.zeros((H, W)), np.zeros((H, W))]
          for j, k in enumerate(order):
            if j >= lag:
              pp, ee, _, _ = ents[order[j - lag]]
              cur[pp] = np.maximum(cur[pp], ee[2])
            p, e, (x0, y0, x1, y1), _ = ents[k]
            res[name][0] += 1
            if cur[p][y0:y1 + 1, x0:x1 + 1].min() >= e[1] * (1 + margin):
              res[name][1] += 1
        for p, e, (x0, y0, x1, y1), _ in ents:
          res["ideal"][0] += 1
          if final[p][y0:y1 + 1, x0:x1 + 1].min() >= e[1] * (1 + margin):
            res["ideal"][1] += 1
  for k, (n, c) in res.items():
    print("%-6s entries %d culled %.1f %%" % (k, n, 100.0 * c / max(n, 1)))
