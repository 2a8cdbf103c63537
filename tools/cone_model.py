"""CPU model of the back-face occlusion test of k_vsd (design study, not product
code). Meshlets (tools/cull_model.py) get a normal cone + bounding sphere; per
(pose, meshlet, tile) entry it counts the back-facing entries and how many of
them are fully occluded by the front-facing ones (rectangle test, exact and at
4 / 8 px block granularity), with the corner bound 1 / zmin.

  python tools/cone_model.py [tuples] [block]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
from bop_toolkit_amd import synth
from oracle import oracle
import cull_model as cm

def cones(pts, faces, ml):
  P = pts.astype(np.float64)
  n = np.cross(P[faces[:,1]]-P[faces[:,0]], P[faces[:,2]]-P[faces[:,0]])
  n /= np.maximum(np.linalg.norm(n, axis=1, keepdims=True), 1e-30)
  cen = P[faces].mean(1)
  if np.sum(((cen - P.mean(0)) * n).sum(1)) < 0: n = -n
  out = []
  for m in ml:
    nn = n[m["tris"]]
    a = nn.mean(0); a /= max(np.linalg.norm(a), 1e-30)
    cosang = np.clip(nn @ a, -1, 1)
    alpha = np.arccos(cosang.min())
    c = m["corners"].mean(0); r = np.linalg.norm(m["corners"] - c, axis=1).max()
    out.append((a, alpha, c, r))
  return out

def is_back(cone, R, t):
  a, alpha, c, r = cone
  if alpha >= np.pi/2: return False
  v = R @ c + t; ac = R @ a
  vn = np.linalg.norm(v)
  va = v @ ac
  s = np.sqrt(max(vn*vn - va*va, 0))
  return va*np.cos(alpha) - s*np.sin(alpha) > r

def main(tuples=12, T=64, blk=4):
  rng = np.random.default_rng(0)
  W, H, K = 640, 480, synth.YCBV_K
  objs = []
  for _ in range(6):
    pts, faces = synth.superellipsoid(50, 100, tuple(rng.uniform(30, 100, 3)), float(rng.uniform(0.5, 1.0)))
    ml = cm.meshlets(pts, faces)
    objs.append((pts, faces, ml, cones(pts, faces, ml)))
  Rg, tg = synth.gt_poses(rng, tuples); Re, te = synth.perturb(rng, Rg, tg)
  st = dict(ent=0, back=0, cull=0, cullblk=0, tri=0, tricull=0, tricullblk=0)
  for i in range(tuples):
    pts, faces, ml, cn = objs[i % 6]
    poses = [(Re[i], te[i]), (Rg[i], tg[i])]
    rects, Q, back = [], [], []
    for R, t in poses:
      bk = [is_back(c, R, t) for c in cn]
      back.append(bk)
      fr = np.concatenate([m["tris"] for m, b in zip(ml, bk) if not b])
      d = oracle.render_depth(pts, faces[fr], R, t, K[0,0], K[1,1], K[0,2], K[1,2], W, H)
      Q.append(np.where(d > 0, 1.0/np.where(d > 0, d, 1), 0.0))
      rects.append([cm.rect_of(m["corners"], R, t, K, W, H) for m in ml])
    rr = [r for rs in rects for r, _ in rs if r is not None]
    rx0, ry0 = min(r[0] for r in rr), min(r[1] for r in rr)
    rx1, ry1 = max(r[2] for r in rr), max(r[3] for r in rr)
    for ty in range(ry0, ry1+1, T):
      for tx in range(rx0, rx1+1, T):
        tx1, ty1 = min(tx+T-1, rx1), min(ty+T-1, ry1)
        for p in range(2):
          # block mins of the phase-A buffer inside the tile
          for mi, (m, (r, qmax)) in enumerate(zip(ml, rects[p])):
            if r is None or r[0] > tx1 or r[2] < tx or r[1] > ty1 or r[3] < ty: continue
            st['ent'] += 1; st['tri'] += len(m["tris"])
            if not back[p][mi]: continue
            st['back'] += 1
            x0, y0, x1, y1 = max(r[0], tx), max(r[1], ty), min(r[2], tx1), min(r[3], ty1)
            thr = qmax*(1+2**-8)
            if Q[p][y0:y1+1, x0:x1+1].min() >= thr:
              st['cull'] += 1; st['tricull'] += len(m["tris"])
            bx0 = tx + (x0-tx)//blk*blk; by0 = ty + (y0-ty)//blk*blk
            bx1 = min(tx + (x1-tx)//blk*blk + blk - 1, tx1); by1 = min(ty + (y1-ty)//blk*blk + blk-1, ty1)
            if Q[p][by0:by1+1, bx0:bx1+1].min() >= thr:
              st['cullblk'] += 1; st['tricullblk'] += len(m["tris"])
  e = st['ent']
  print({k: (v, round(100*v/ (e if not k.startswith('tri') else st['tri']),1)) for k,v in st.items()})

if __name__ == '__main__':
  main(int(sys.argv[1]) if len(sys.argv) > 1 else 12, blk=int(sys.argv[2]) if len(sys.argv) > 2 else 4)
