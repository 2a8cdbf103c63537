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


def _workload(seed, n_img=6, ks=(1, 3, 5), W=640, H=480, meshes=((30, 60), (50, 100))):
  import torch
  from bop_toolkit_amd import synth
  from bop_toolkit_amd.batch import BatchEvaluator
  rng = np.random.default_rng(seed)
  ev = BatchEvaluator(0)
  objs = []
  for o, (nl, nn) in enumerate(meshes):
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


@pytest.mark.parametrize("big", [(90, 140), (130, 150)])
def test_shared_renders_large_meshes(oracle_mod, big):
  """Largest object of the context with >= 394 / >= 610 meshlets (25.2k / 39k
  triangles): the render mode holds one pose's meshlet rectangles (1 / 2 per
  thread) where the fused kernel holds both poses' (2 / 4 per thread); the
  results are the same bits."""
  import torch
  from bop_toolkit_amd.batch import unique_renders
  ev, objs, obj, fi, pe, pg, fr, cam, dia, t = _workload(55, n_img=3, ks=(2, 3),
                                                        meshes=(big, (30, 60)))
  nf = len(objs[0][1])
  assert (256 < nf / 64 <= 512) if big == (90, 140) else (512 < nf / 64 <= 1024)
  n = len(obj)
  ro, rp, rf, er, gr = unique_renders(obj, pe, pg, fi)
  taus = np.arange(0.05, 0.51, 0.05)
  fused = ev.vsd(ev.slots(obj), t(pe, torch.float64), t(pg, torch.float64), t(fi, torch.int32),
                 t(fr, torch.float32), t(cam, torch.float64), 15.0, taus,
                 t(dia, torch.float64)).cpu().numpy()
  shared = ev.vsd_shared(ev.slots(ro), t(rp, torch.float64), t(rf, torch.int32),
                         t(er, torch.int32), t(gr, torch.int32), t(fr, torch.float32),
                         t(cam, torch.float64), 15.0, taus, t(dia, torch.float64)).cpu().numpy()
  assert np.ptp(fused) > 0.1
  assert np.array_equal(shared, fused)
  K = cam[0]
  for i in range(0, n, 5):
    pts, faces = objs[obj[i]]
    de = oracle_mod.render_depth(pts, faces, pe[i, :9].reshape(3, 3), pe[i, 9:], *K, 640, 480)
    dg = oracle_mod.render_depth(pts, faces, pg[i, :9].reshape(3, 3), pg[i, 9:], *K, 640, 480)
    assert list(shared[i]) == oracle_mod.vsd_depths(fr[fi[i]], de, dg, *K, 15.0, taus, True,
                                                    dia[i], "step"), i


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


def test_shared_dev_zero_renders_refused():
  """n > 0 tuples with no renders used to return OK with the output
  unwritten; it is refused now (nothing could be indexed)."""
  import torch
  ev, objs, obj, fi, pe, pg, fr, cam, dia, t = _workload(53, n_img=1, ks=(1,))
  e = torch.zeros(2, dtype=torch.int32, device=ev.device)
  with pytest.raises(ValueError):
    ev.vsd_shared(ev.slots([]), t(np.zeros((0, 12)), torch.float64), t([], torch.int32), e, e,
                  t(fr, torch.float32), t(cam, torch.float64), 15.0,
                  np.arange(0.05, 0.51, 0.05), t(dia[:2], torch.float64))


@pytest.mark.parametrize("ntau", [10, 23])
def test_unions_flag_batch_api(ntau):
  """BOPX_VSD_UNIONS through BatchEvaluator gets its own n slots
  (no write past the tensor): (vsd, unions) returned, vsd equal to the call
  without the flag, the same unions from the fused and the shared path, and a
  too-small caller-supplied out is refused."""
  import torch
  from bop_toolkit_amd import _lib
  from bop_toolkit_amd.batch import unique_renders
  ev, objs, obj, fi, pe, pg, fr, cam, dia, t = _workload(55, n_img=3)
  taus = np.linspace(0.02, 0.6, ntau)
  n = len(obj)
  args = (ev.slots(obj), t(pe, torch.float64), t(pg, torch.float64), t(fi, torch.int32),
          t(fr, torch.float32), t(cam, torch.float64), 15.0, taus, t(dia, torch.float64))
  plain = ev.vsd(*args).cpu().numpy()
  guard = torch.full((n * ntau + n + 64,), 7.0, dtype=torch.float64, device=ev.device)
  v, u = ev.vsd(*args, out=guard, delta_flags=_lib.VSD_UNIONS)
  assert np.array_equal(v.cpu().numpy(), plain)
  assert (guard[n * ntau + n:] == 7.0).all()  # nothing written past the unions
  un = u.cpu().numpy()
  assert (un >= 0).all() and (un > 0).any()
  assert np.array_equal(plain[un == 0], np.ones_like(plain[un == 0]))
  ro, rp, rf, er, gr = unique_renders(obj, pe, pg, fi)
  vs, us = ev.vsd_shared(ev.slots(ro), t(rp, torch.float64), t(rf, torch.int32),
                         t(er, torch.int32), t(gr, torch.int32), t(fr, torch.float32),
                         t(cam, torch.float64), 15.0, taus, t(dia, torch.float64),
                         delta_flags=_lib.VSD_UNIONS)
  assert np.array_equal(vs.cpu().numpy(), plain) and np.array_equal(us.cpu().numpy(), un)
  with pytest.raises(ValueError):
    ev.vsd(*args, out=torch.empty((n, ntau), dtype=torch.float64, device=ev.device),
           delta_flags=_lib.VSD_UNIONS)


def test_shared_wide_image_column_blocks(oracle_mod):
  """Unions wider than k_vsd_pair's 1,024-column LDS block (4,096 x 512
  image, estimates shifted right by up to ~3,700 px, one partly off the right
  edge): equal to the fused kernel bit for bit and to the oracle."""
  import torch
  from bop_toolkit_amd import synth
  from bop_toolkit_amd.batch import BatchEvaluator, unique_renders
  rng = np.random.default_rng(54)
  W, H = 4096, 512
  ev = BatchEvaluator(0)
  pts, faces = synth.superellipsoid(30, 60, (60.0, 45.0, 50.0), 0.7)
  ev.add_object(0, pts, faces)
  K = np.array([[1075.0, 0.0, 400.0], [0.0, 1075.0, 256.0], [0.0, 0.0, 1.0]])
  Rg, tg = synth.gt_poses(rng, 2, z_range=(650.0, 750.0), xy=(60.0, 40.0))
  gts = [np.concatenate([Rg[i].reshape(9), tg[i]]) for i in range(2)]
  ests = []
  for dx in (0.0, 800.0, 1600.0, 2600.0, None):
    Re, te = synth.perturb(rng, Rg[:1], tg[:1], outlier_frac=0.0)
    te = te.copy()
    if dx is None:  # centre 20 px left of the right edge: the render is cut by it
      dx = (W - 20 - K[0, 2]) * te[0, 2] / K[0, 0] - te[0, 0]
    te[0, 0] += dx
    ests.append(np.concatenate([Re[0].reshape(9), te[0]]))
  pe = np.stack([e for e in ests for _ in gts])
  pg = np.stack([g for _ in ests for g in gts])
  n = len(pe)
  obj = np.zeros(n, np.int32)
  fi = np.zeros(n, np.int32)
  cam = np.array([[K[0, 0], K[1, 1], K[0, 2], K[1, 2]]])
  dev = ev.device
  t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
  frames = ev.render(ev.slots([0, 0]), t(np.stack(gts), torch.float64), t([0, 0], torch.int32),
                     t(cam, torch.float64), 1, W, H)
  fr = frames.cpu().numpy()
  fr = np.where(fr > 0, fr, 1500.0)
  fr = np.round(fr + rng.normal(0.0, 3.0, fr.shape)).astype(np.float32)
  fr[rng.random(fr.shape) < 0.1] = 0.0
  dia = np.full(n, 150.0)
  taus = np.arange(0.05, 0.51, 0.05)
  ro, rp, rf, er, gr = unique_renders(obj, pe, pg, fi)
  fused = ev.vsd(ev.slots(obj), t(pe, torch.float64), t(pg, torch.float64), t(fi, torch.int32),
                 t(fr, torch.float32), t(cam, torch.float64), 15.0, taus,
                 t(dia, torch.float64)).cpu().numpy()
  shared = ev.vsd_shared(ev.slots(ro), t(rp, torch.float64), t(rf, torch.int32),
                         t(er, torch.int32), t(gr, torch.int32), t(fr, torch.float32),
                         t(cam, torch.float64), 15.0, taus, t(dia, torch.float64)).cpu().numpy()
  assert np.array_equal(shared, fused)
  assert (fused[-4:] == 1.0).all() and (fused[:2] < 1.0).any()  # shifted estimates miss
  for i in range(n):
    de = oracle_mod.render_depth(pts, faces, pe[i, :9].reshape(3, 3), pe[i, 9:], *cam[0], W, H)
    dg = oracle_mod.render_depth(pts, faces, pg[i, :9].reshape(3, 3), pg[i, 9:], *cam[0], W, H)
    if i == n - 1:
      assert (de[:, W - 1] > 0).any() and (de[:, 0] == 0).all()  # cut by the right edge
    assert list(shared[i]) == oracle_mod.vsd_depths(fr[0], de, dg, *cam[0], 15.0, taus, True,
                                                    dia[i], "step"), i
