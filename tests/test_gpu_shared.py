"""Shared renders for multi-instance images (k_vsd render mode + k_vsd_pair)
against the fused per-tuple k_vsd and the oracle.

The reference evaluates every estimate against every GT instance of its object
(eval_calc_errors.py:281-290) and renders both poses per tuple
(pose_error.py:42-45): k instances and k estimates cost 2k^2 renders. The
shared path renders each distinct pose once; its VSD must be the fused
kernel's bit for bit (step cost), the tlinear sums within 1e-13.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _workload(seed, n_img=6, ks=(1, 3, 5), W=640, H=480):
  import torch
  from bop_toolkit_amd import synth
  from bop_toolkit_amd.batch import BatchEvaluator
  rng = np.random.default_rng(seed)
  ev = BatchEvaluator(0)
  objs = []
  for o, (nl, nn) in enumerate([(30, 60), (50, 100)]):
    pts, faces = synth.superellipsoid(nl, nn, tuple(rng.uniform(35.0, 70.0, 3)), 0.7)
    ev.add_object(o, pts, faces)
    objs.append((pts, faces))
  K = synth.YCBV_K
  inst = []  # (frame, obj, gt pose) of every GT instance
  for f in range(n_img):
    for o in range(2):
      k = ks[(f + o) % len(ks)]
      Rg, tg = synth.gt_poses(rng, k, z_range=(600.0, 1100.0), xy=(140.0, 100.0))
      for i in range(k):
        inst.append((f, o, np.concatenate([Rg[i].reshape(9), tg[i]])))
  # tuples: every estimate x every GT of its object in its image
  tup_obj, tup_f, pe, pg = [], [], [], []
  for f in range(n_img):
    for o in range(2):
      gts = [p for (ff, oo, p) in inst if ff == f and oo == o]
      k = len(gts)
      Rg = np.stack([g[:9].reshape(3, 3) for g in gts])
      tg = np.stack([g[9:] for g in gts])
      Re, te = synth.perturb(rng, Rg, tg)
      ests = [np.concatenate([Re[i].reshape(9), te[i]]) for i in range(k)]
      if k >= 3:
        ests[0] = gts[1].copy()  # an estimate equal to a GT: one shared render
        ests[1][11] = -300.0  # behind the camera: empty ROI
        ests[2][9] += 5000.0  # far off-screen
      for e in ests:
        for g in gts:
          tup_obj.append(o)
          tup_f.append(f)
          pe.append(e)
          pg.append(g)
  n = len(tup_obj)
  obj = np.array(tup_obj, np.int32)
  fi = np.array(tup_f, np.int32)
  pe, pg = np.stack(pe), np.stack(pg)
  cam = np.tile([K[0, 0], K[1, 1], K[0, 2], K[1, 2]], (n_img, 1)).astype(np.float64)
  dev = ev.device
  t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
  ig = np.array([p for (_, _, p) in inst])
  frames = ev.render(ev.slots([o for (_, o, _) in inst]), t(ig, torch.float64),
                     t([f for (f, _, _) in inst], torch.int32), t(cam, torch.float64), n_img, W, H)
  frames = torch.where(frames > 0, frames, torch.full_like(frames, 1500.0))
  fr = frames.cpu().numpy()
  fr = np.round(fr + rng.normal(0.0, 3.0, fr.shape)).astype(np.float32)
  fr[rng.random(fr.shape) < 0.1] = 0.0
  dia = np.array([140.0, 180.0])[obj]
  return ev, objs, obj, fi, pe, pg, fr, cam, dia, t


@pytest.mark.parametrize("cost,taus", [("step", np.arange(0.05, 0.51, 0.05)),
                                       ("step", list(np.arange(0.05, 0.51, 0.05)) + [0.7, 0.0,
                                                                                     1e-3]),
                                       ("tlinear", np.arange(0.05, 0.51, 0.05))])
def test_shared_renders_equal_fused(oracle_mod, cost, taus):
  import torch
  from bop_toolkit_amd.batch import unique_renders
  ev, objs, obj, fi, pe, pg, fr, cam, dia, t = _workload(51)
  n = len(obj)
  ro, rp, rf, er, gr = unique_renders(obj, pe, pg, fi)
  assert len(ro) < 2 * n  # renders are shared
  taus = np.asarray(taus, np.float64)
  fused = ev.vsd(ev.slots(obj), t(pe, torch.float64), t(pg, torch.float64), t(fi, torch.int32),
                 t(fr, torch.float32), t(cam, torch.float64), 15.0, taus,
                 t(dia, torch.float64), cost_type=cost).cpu().numpy()
  shared = ev.vsd_shared(ev.slots(ro), t(rp, torch.float64), t(rf, torch.int32),
                         t(er, torch.int32), t(gr, torch.int32), t(fr, torch.float32),
                         t(cam, torch.float64), 15.0, taus, t(dia, torch.float64),
                         cost_type=cost).cpu().numpy()
  assert np.ptp(fused) > 0.1
  if cost == "step":
    assert np.array_equal(shared, fused)
  else:
    np.testing.assert_allclose(shared, fused, rtol=0, atol=1e-13)
  # a subsample against the oracle raster + VSD
  K = cam[0]
  for i in range(0, n, 7):
    pts, faces = objs[obj[i]]
    de = oracle_mod.render_depth(pts, faces, pe[i, :9].reshape(3, 3), pe[i, 9:], *K, 640, 480)
    dg = oracle_mod.render_depth(pts, faces, pg[i, :9].reshape(3, 3), pg[i, 9:], *K, 640, 480)
    ref = oracle_mod.vsd_depths(fr[fi[i]], de, dg, *K, 15.0, taus, True, dia[i], cost)
    if cost == "step":
      assert list(shared[i]) == ref, i
    else:
      np.testing.assert_allclose(shared[i], ref, rtol=0, atol=1e-12)


def test_shared_host_entry_unions_and_checks(oracle_mod):
  """bopx_vsd_shared_batch (host buffers) with BOPX_VSD_UNIONS and a float64
  delta: the same errors and union counts as bopx_vsd_batch; bad render
  indices and mismatched frames are refused."""
  from bop_toolkit_amd import _lib
  from bop_toolkit_amd._lib import _d, _f, _i32, ptr
  from bop_toolkit_amd.batch import unique_renders
  ev, objs, obj, fi, pe, pg, fr, cam, dia, t = _workload(52, n_img=3, ks=(3, 4))
  n = len(obj)
  ro, rp, rf, er, gr = unique_renders(obj, pe, pg, fi)
  taus = np.arange(0.05, 0.51, 0.05)
  flags = _lib.DELTA_F64 | _lib.VSD_UNIONS
  c = ev.ctx
  a = np.empty(n * 10 + n)
  c.call("bopx_vsd_batch", n, ptr(obj, _i32), ptr(pe, _d), ptr(pg, _d), ptr(fi, _i32),
         ptr(fr, _f), len(fr), 640, 480, ptr(cam, _d), 15.3, flags, ptr(taus, _d), 10, 1,
         ptr(dia, _d), 0, ptr(a, _d))
  b = np.empty(n * 10 + n)
  c.call("bopx_vsd_shared_batch", len(ro), ptr(ro, _i32), ptr(rp, _d), ptr(rf, _i32), n,
         ptr(er, _i32), ptr(gr, _i32), ptr(fr, _f), len(fr), 640, 480, ptr(cam, _d), 15.3, flags,
         ptr(taus, _d), 10, 1, ptr(dia, _d), 0, ptr(b, _d))
  assert np.array_equal(a, b)
  assert (a[n * 10:] > 0).all() and np.ptp(a[n * 10:]) > 0  # union counts (GT always visible)
  bad = gr.copy()
  bad[0] = len(ro)
  with pytest.raises(ValueError):
    c.call("bopx_vsd_shared_batch", len(ro), ptr(ro, _i32), ptr(rp, _d), ptr(rf, _i32), n,
           ptr(er, _i32), ptr(bad, _i32), ptr(fr, _f), len(fr), 640, 480, ptr(cam, _d), 15.0, 0,
           ptr(taus, _d), 10, 1, ptr(dia, _d), 0, ptr(b, _d))
  rf2 = rf.copy()
  rf2[er[0]] = (rf2[er[0]] + 1) % len(fr)
  with pytest.raises(ValueError):
    c.call("bopx_vsd_shared_batch", len(ro), ptr(ro, _i32), ptr(rp, _d), ptr(rf2, _i32), n,
           ptr(er, _i32), ptr(gr, _i32), ptr(fr, _f), len(fr), 640, 480, ptr(cam, _d), 15.0, 0,
           ptr(taus, _d), 10, 1, ptr(dia, _d), 0, ptr(b, _d))


def test_shared_dev_bad_index_gives_nan():
  """The _dev entry cannot check render indices on the host: an index past
  the render list gives NaN errors for that tuple (and no out-of-bounds read)."""
  import torch
  from bop_toolkit_amd.batch import unique_renders
  ev, objs, obj, fi, pe, pg, fr, cam, dia, t = _workload(53, n_img=2, ks=(2,))
  ro, rp, rf, er, gr = unique_renders(obj, pe, pg, fi)
  gr = gr.copy()
  gr[1] = 1 << 20
  out = ev.vsd_shared(ev.slots(ro), t(rp, torch.float64), t(rf, torch.int32),
                      t(er, torch.int32), t(gr, torch.int32), t(fr, torch.float32),
                      t(cam, torch.float64), 15.0, np.arange(0.05, 0.51, 0.05),
                      t(dia, torch.float64)).cpu().numpy()
  assert np.isnan(out[1]).all() and np.isfinite(out[0]).all()
