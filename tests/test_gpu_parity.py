"""HIP path vs the oracle / golden vectors, through the C-ABI (libbopx.so).

Bars (BASELINE.json north_star): bit-exact for masks, counts, raster depth,
distance images and VSD; within 1e-4 mm / 1e-4 px for MSSD/MSPD/ADD/ADI/PROJ
(observed ~1e-12)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-4


@pytest.fixture(scope="module")
def ctx():
  from bop_toolkit_amd import _lib
  return _lib.Context(0)


@pytest.fixture(scope="module")
def golden_ctx(ctx, golden_errors):
  g = golden_errors
  for o in range(4):
    ctx.add_object(100 + o, g["pts_%d" % o], g["faces_%d" % o])
    ctx.set_symmetries(100 + o, g["syms_%d" % o])
  return ctx


def _batch(ctx, name, ids, pe, pg, K=None):
  from bop_toolkit_amd._lib import _d, _i32, ptr
  ids = np.ascontiguousarray(ids, np.int32)
  pe = np.ascontiguousarray(pe, np.float64)
  pg = np.ascontiguousarray(pg, np.float64)
  out = np.empty(len(ids))
  if K is None:
    ctx.call(name, len(ids), ptr(ids, _i32), ptr(pe, _d), ptr(pg, _d), ptr(out, _d))
  else:
    K = np.ascontiguousarray(K, np.float64)
    ctx.call(name, len(ids), ptr(ids, _i32), ptr(pe, _d), ptr(pg, _d), ptr(K, _d), ptr(out, _d))
  return out


@pytest.mark.parametrize("name", ["mssd", "mspd", "add", "adi", "proj"])
def test_point_errors_vs_golden(golden_ctx, golden_errors, name):
  g = golden_errors
  ids = g["obj"] + 100
  K = g["K"] if name in ("mspd", "proj") else None
  out = _batch(golden_ctx, "bopx_%s_batch" % name, ids, g["pose_est"], g["pose_gt"], K)
  np.testing.assert_allclose(out, g["out_" + name], rtol=0, atol=TOL)
  # scale-aware: float64 rounding only
  assert np.max(np.abs(out - g["out_" + name]) / np.maximum(1.0, np.abs(g["out_" + name]))) < 1e-9


def test_drop_in_point_errors(golden_errors):
  from bop_toolkit_amd import pose_error as pe
  g = golden_errors
  for i in range(0, len(g["obj"]), 3):
    o = int(g["obj"][i])
    pts = g["pts_%d" % o]
    syms = [{"R": s[:9].reshape(3, 3), "t": s[9:].reshape(3, 1)} for s in g["syms_%d" % o]]
    Re, te_ = g["pose_est"][i][:9].reshape(3, 3), g["pose_est"][i][9:].reshape(3, 1)
    Rg, tg = g["pose_gt"][i][:9].reshape(3, 3), g["pose_gt"][i][9:].reshape(3, 1)
    K = g["K"][i].reshape(3, 3)
    assert abs(pe.mssd(Re, te_, Rg, tg, pts, syms) - g["out_mssd"][i]) < TOL
    assert abs(pe.mspd(Re, te_, Rg, tg, K, pts, syms) - g["out_mspd"][i]) < TOL
    assert abs(pe.add(Re, te_, Rg, tg, pts) - g["out_add"][i]) < TOL
    assert abs(pe.adi(Re, te_, Rg, tg, pts) - g["out_adi"][i]) < TOL
    assert abs(pe.proj(Re, te_, Rg, tg, K, pts) - g["out_proj"][i]) < TOL


def test_drop_in_cache_bounded(golden_errors, monkeypatch):
  """Fresh arrays per call (model['pts'] * 1.0) share one content-keyed HBM slot,
  and distinct point sets beyond the LRU bound evict (and free) old slots."""
  from bop_toolkit_amd import pose_error as pe
  from bop_toolkit_amd import runtime
  g = golden_errors
  pts = g["pts_0"]
  Re, te_ = g["pose_est"][0][:9].reshape(3, 3), g["pose_est"][0][9:].reshape(3, 1)
  Rg, tg = g["pose_gt"][0][:9].reshape(3, 3), g["pose_gt"][0][9:].reshape(3, 1)
  want = pe.add(Re, te_, Rg, tg, pts)
  n0 = runtime.resident_count()
  for _ in range(50):
    assert pe.add(Re, te_, Rg, tg, pts * 1.0) == want
  assert runtime.resident_count() <= n0 + 1
  monkeypatch.setattr(runtime, "MAX_RESIDENT", 8)
  monkeypatch.setattr(runtime, "MAX_IDENTITY", 32)
  for k in range(40):
    shifted = pts + float(k + 1)
    got = pe.add(Re, te_, Rg, tg, shifted)
    assert abs(got - pe.add(Re, te_, Rg, tg, shifted.copy())) == 0.0
    assert runtime.resident_count() <= 8
  assert pe.add(Re, te_, Rg, tg, pts) == want


def test_visibility_numpy_scalar_delta_float32(oracle_mod):
  """delta = np.float64(15.3): compared in float32 (legacy NumPy casting of the
  reference's runtime, runtime.delta_flags), so d_diff = float32(15.3) is visible."""
  from bop_toolkit_amd import visibility
  rng = np.random.default_rng(7)
  dt = np.round(rng.uniform(400, 900, (48, 64)) * 64) / 64
  d15 = float(np.float32(15.3))
  dm = dt + np.where(rng.random(dt.shape) < 0.5, d15, 16.0)
  dm[::5] = 0.0
  dt[1::7] = 0.0
  got = visibility.estimate_visib_mask_gt(dt, dm, np.float64(15.3))
  want = oracle_mod.visib_mask(dt, dm, 15.3, delta_f64=False).astype(bool)
  assert np.array_equal(got, want)
  assert got[(dm - dt == d15) & (dm > 0)].all()


def test_dist_and_visibility_bit_exact(golden_vsd):
  from bop_toolkit_amd import misc, visibility
  g = golden_vsd
  for i in range(3):
    dt = misc.depth_im_to_dist_im_fast(g["depth_test"][i], g["K"])
    dgt = misc.depth_im_to_dist_im_fast(g["depth_gt"][i], g["K"])
    de = misc.depth_im_to_dist_im_fast(g["depth_est"][i], g["K"])
    assert np.array_equal(dt, g["dist_test_%d" % i])
    assert np.array_equal(dgt, g["dist_gt_%d" % i])
    assert np.array_equal(de, g["dist_est_%d" % i])
    vg = visibility.estimate_visib_mask_gt(dt, dgt, 15.0, visib_mode="bop19")
    ve = visibility.estimate_visib_mask_est(dt, de, vg, 15.0, visib_mode="bop19")
    vg18 = visibility.estimate_visib_mask_gt(dt, dgt, 15.0, visib_mode="bop18")
    assert np.array_equal(np.packbits(vg), g["visib_gt_%d" % i])
    assert np.array_equal(np.packbits(ve), g["visib_est_%d" % i])
    assert np.array_equal(np.packbits(vg18), g["visib_gt18_%d" % i])
  with pytest.raises(ValueError):
    visibility.estimate_visib_mask_gt(dt, dgt, 15.0, visib_mode="bop17")


class _Stub:
  def __init__(self, maps):
    self.maps = list(maps)

  def render_object(self, obj_id, R, t, fx, fy, cx, cy):
    return {"depth": self.maps.pop(0)}


def test_vsd_foreign_renderer_bit_exact(golden_vsd):
  from bop_toolkit_amd import pose_error as pe
  g = golden_vsd
  K, taus = g["K"], list(g["taus"])
  I, z = np.eye(3), np.zeros((3, 1))
  for i in range(len(g["vsd_step"])):
    de, dg, dt = g["depth_est"][i], g["depth_gt"][i], g["depth_test"][i]
    r = pe.vsd(I, z, I, z, dt, K, 15.0, taus, True, 120.0, _Stub([de, dg]), 1, "step")
    assert r == list(g["vsd_step"][i])
    r = pe.vsd(I, z, I, z, dt, K, 15.0, [5.0, 10.0, 20.0], False, 120.0, _Stub([de, dg]), 1)
    assert r == list(g["vsd_step_raw"][i])
    r = pe.vsd(I, z, I, z, dt, K, 5.0, taus, True, 120.0, _Stub([de, dg]), 1)
    assert r == list(g["vsd_delta5"][i])
    r = pe.vsd(I, z, I, z, dt, K, 15.0, taus, True, 120.0, _Stub([de, dg]), 1, "tlinear")
    np.testing.assert_allclose(r, g["vsd_tlinear"][i], rtol=0, atol=1e-12)
  zz = np.zeros_like(g["depth_test"][0])
  assert pe.vsd(I, z, I, z, g["depth_test"][0], K, 15.0, taus, True, 120.0, _Stub([zz, zz]), 1,
                "bogus") == list(g["vsd_empty"])
  with pytest.raises(ValueError):
    pe.vsd(I, z, I, z, g["depth_test"][3], K, 15.0, taus, True, 120.0,
           _Stub([g["depth_est"][3], g["depth_gt"][3]]), 1, "bogus")


def _scene(seed, n, W=640, H=480, n_lat=20, n_lon=40, K=None, xy=(150.0, 100.0),
           z_range=(450.0, 1200.0), mesh=None):
  from bop_toolkit_amd import synth
  rng = np.random.default_rng(seed)
  pts, faces = (synth.superellipsoid(n_lat, n_lon, (45.0, 35.0, 55.0), 0.7) if mesh is None
                else mesh)
  Rg, tg = synth.gt_poses(rng, n, z_range=z_range, xy=xy)
  Re, te_ = synth.perturb(rng, Rg, tg)
  K = synth.LMO_K if K is None else K
  return rng, pts, faces, Rg, tg, Re, te_, K


def test_raster_bit_exact_vs_oracle(ctx, oracle_mod):
  from bop_toolkit_amd.renderer import create_renderer
  rng, pts, faces, Rg, tg, Re, te_, K = _scene(7, 24)
  ren = create_renderer(640, 480, "hip", mode="depth")
  ren.add_object_arrays(5, pts, faces)
  fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
  for i in range(24):
    R, t = (Re[i], te_[i]) if i % 2 else (Rg[i], tg[i])
    if i == 3:
      t = np.array([0.0, 0.0, 60.0])  # very close: vertices beyond the guard band
    if i == 4:
      t = np.array([0.0, 0.0, -200.0])  # behind the camera
    d_hip = ren.render_object(5, R, t, fx, fy, cx, cy)["depth"]
    d_ref = oracle_mod.render_depth(pts, faces, R, t, fx, fy, cx, cy, 640, 480)
    assert np.array_equal(d_hip, d_ref), i
    if i not in (3, 4):
      assert (d_hip > 0).sum() > 100


def _fused_vs_oracle(oracle_mod, seed, n, W, H, K, n_lat, n_lon, delta=15.0, cost="step",
                     normalized=True, taus=None, dia=None, delta_f64=False, **scene):
  """Fused k_vsd (raster + VSD) vs oracle raster + oracle VSD, bit for bit."""
  from bop_toolkit_amd import _lib
  from bop_toolkit_amd._lib import _d, _f, _i32, ptr
  rng, pts, faces, Rg, tg, Re, te_, _ = _scene(seed, n, W, H, n_lat, n_lon, **scene)
  ctx = _lib.Context(0)
  ctx.add_object(9, pts, faces)
  fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
  frames = []
  for i in range(n):
    dg = oracle_mod.render_depth(pts, faces, Rg[i], tg[i], fx, fy, cx, cy, W, H)
    dt = np.where(dg > 0, dg, 1600.0).astype(np.float32)
    dt += rng.normal(0, 3.0, dt.shape).astype(np.float32)
    dt[rng.random(dt.shape) < 0.1] = 0.0
    frames.append(np.round(dt).astype(np.float32))
  frames = np.stack(frames)
  taus = np.arange(0.05, 0.51, 0.05) if taus is None else np.asarray(taus, np.float64)
  ids = np.full(n, 9, np.int32)
  pe = np.concatenate([Re.reshape(n, 9), te_], 1)
  pg = np.concatenate([Rg.reshape(n, 9), tg], 1)
  fi = np.arange(n, dtype=np.int32)
  cam = np.tile([fx, fy, cx, cy], (n, 1)).astype(np.float64)
  dia = np.full(n, 160.0) if dia is None else np.asarray(dia, np.float64)
  out = np.empty((n, len(taus)))
  code = {"step": 0, "tlinear": 1}[cost]
  ctx.call("bopx_vsd_batch", n, ptr(ids, _i32), ptr(pe, _d), ptr(pg, _d), ptr(fi, _i32),
           ptr(frames, _f), n, W, H, ptr(cam, _d), delta, int(delta_f64), ptr(taus, _d), len(taus),
           int(normalized), ptr(dia, _d), code, ptr(out, _d))
  for i in range(n):
    de = oracle_mod.render_depth(pts, faces, Re[i], te_[i], fx, fy, cx, cy, W, H)
    dg = oracle_mod.render_depth(pts, faces, Rg[i], tg[i], fx, fy, cx, cy, W, H)
    ref = oracle_mod.vsd_depths(frames[i], de, dg, fx, fy, cx, cy, delta, taus, normalized,
                                dia[i], cost, delta_f64)
    if cost == "step":
      assert list(out[i]) == ref, (i, out[i], ref)
    else:
      np.testing.assert_allclose(out[i], ref, rtol=0, atol=1e-12)
  ctx.close()
  return out


def test_fused_vsd_tile_parallel_matches_one_workgroup():
  """Tile-parallel mode (kern_vsd.hip vsd_split: batches below 1,024 tuples split
  each tuple's ROI tiles over up to 16 workgroups, k_vsd_combine sums the rows)
  against the one-workgroup-per-tuple launch of a 1,100-tuple batch: step cost
  bit-identical, tlinear within 1e-13 (its float64 sums change order), the
  silhouette cover mode bit-identical."""
  from bop_toolkit_amd import _lib, synth
  from bop_toolkit_amd._lib import _d, _f, _i32, ptr
  n, nf, W, H = 1100, 8, 640, 480
  rng, pts, faces, Rg, tg, Re, te_, K = _scene(41, n, n_lat=30, n_lon=60,
                                              z_range=(330.0, 900.0))
  ctx = _lib.Context(0)
  ctx.add_object(3, pts, faces)
  fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
  frames = np.round(rng.uniform(300.0, 1300.0, (nf, H, W))).astype(np.float32)
  frames[rng.random(frames.shape) < 0.1] = 0.0
  taus = np.arange(0.05, 0.51, 0.05)
  ids = np.full(n, 3, np.int32)
  pe = np.concatenate([Re.reshape(n, 9), te_], 1)
  pg = np.concatenate([Rg.reshape(n, 9), tg], 1)
  fi = (np.arange(n) % nf).astype(np.int32)
  cam = np.tile([fx, fy, cx, cy], (nf, 1)).astype(np.float64)
  dia = np.full(n, 150.0)

  def run(lo, hi, code):
    m = hi - lo
    out = np.empty((m, len(taus)))
    ctx.call("bopx_vsd_batch", m, ptr(ids[lo:hi], _i32), ptr(pe[lo:hi].copy(), _d),
             ptr(pg[lo:hi].copy(), _d), ptr(fi[lo:hi].copy(), _i32), ptr(frames, _f), nf, W, H,
             ptr(cam, _d), 15.0, 0, ptr(taus, _d), len(taus), 1, ptr(dia[lo:hi].copy(), _d),
             code, ptr(out, _d))
    return out

  for code in (0, 1):
    full = run(0, n, code)
    assert np.ptp(full) > 0.1
    # splits 16, 16, 13 and 4 workgroups per tuple
    parts = [run(0, 1, code), run(1, 25, code), run(25, 100, code), run(100, 400, code)]
    got = np.concatenate(parts)
    if code == 0:
      assert np.array_equal(got, full[:400])
    else:
      np.testing.assert_allclose(got, full[:400], rtol=0, atol=1e-13)
  # silhouette cover mode (bboxes min / max over the splits, counts summed)
  def cover(lo, hi):
    out = np.empty((hi - lo, 10))
    ctx.call("bopx_cover_batch", hi - lo, ptr(ids[lo:hi], _i32), ptr(pe[lo:hi].copy(), _d),
             ptr(pg[lo:hi].copy(), _d), ptr(fi[lo:hi].copy(), _i32), nf, W, H, ptr(cam, _d),
             ptr(out, _d))
    return out
  full = cover(0, n)
  assert (full[:, 0] > 0).all()
  got = np.concatenate([cover(0, 1), cover(1, 25), cover(25, 100), cover(100, 400)])
  assert np.array_equal(got, full[:400])

  # GT-info mode on the calc_gt_info canvas (3x the image, calc_gt_info.py:66-73)
  def gt_info(lo, hi):
    out = np.empty((hi - lo, 11))
    ctx.call("bopx_gt_info_batch", hi - lo, ptr(ids[lo:hi], _i32), ptr(pg[lo:hi].copy(), _d),
             ptr(fi[lo:hi].copy(), _i32), ptr(frames, _f), nf, W, H, ptr(cam, _d), 15.0, 0, 3,
             ptr(out, _d), None)
    return out
  full = gt_info(0, n)
  assert (full[:, 0] > 0).all() and (full[:, 1] > 0).any()
  got = np.concatenate([gt_info(0, 1), gt_info(1, 25), gt_info(25, 100), gt_info(100, 400)])
  assert np.array_equal(got, full[:400])
  ctx.close()


def test_fused_vsd_bit_exact_lmo(oracle_mod):
  from bop_toolkit_amd import synth
  out = _fused_vs_oracle(oracle_mod, 11, 40, 640, 480, synth.LMO_K, 30, 60)
  assert np.ptp(out) > 0.1  # non-trivial errors


def test_fused_vsd_bit_exact_ycbv_big_mesh(oracle_mod):
  from bop_toolkit_amd import synth
  _fused_vs_oracle(oracle_mod, 12, 16, 640, 480, synth.YCBV_K, 50, 100)


def test_fused_vsd_tlinear_and_raw(oracle_mod):
  from bop_toolkit_amd import synth
  _fused_vs_oracle(oracle_mod, 13, 12, 640, 480, synth.LMO_K, 20, 40, cost="tlinear")
  _fused_vs_oracle(oracle_mod, 14, 12, 720, 540, synth.TLESS_K, 20, 40, delta=5.0,
                   normalized=False)


def test_fused_vsd_bit_exact_image_borders(oracle_mod):
  """Objects straddling and leaving the image borders: ROIs clipped at the
  image edge, tiles cut by the ROI (the row walk's unmasked column past a cut,
  cleared by the pixel compaction, must not leak into later tiles)."""
  from bop_toolkit_amd import synth
  out = _fused_vs_oracle(oracle_mod, 31, 48, 640, 480, synth.LMO_K, 24, 48, xy=(420.0, 320.0),
                         z_range=(420.0, 800.0))
  assert np.ptp(out) > 0.1


def test_fused_vsd_step_thresholds_edge_cases(oracle_mod):
  """Per-tuple step thresholds (kern_vsd.hip step_threshold) and the float32
  visibility threshold (runtime.cpp visib_thr32) vs the oracle's per-pixel
  division and comparison, on diameters and taus at and beyond the edges:
  tiny, huge, zero, signed zero, negative, infinite and NaN diameters; zero,
  negative, subnormal, huge, infinite and NaN taus; float64 delta."""
  from bop_toolkit_amd import synth
  inf, nan = float("inf"), float("nan")
  dia = [160.0, 1e-300, 1e300, 0.0, -0.0, -160.0, inf, -inf, nan, 3.3e-5, 7.0,
         np.nextafter(160.0, inf), 95.123456789, 1.0]
  n = len(dia)
  bop = list(np.arange(0.05, 0.51, 0.05))
  # 10 taus: the NT = 10 kernel; 13 taus: the NT = 16 kernel
  taus10 = [0.0, -0.1, 5e-324, 1e308, inf, -inf, 0.1, 0.35, 2.0, 0.15000000000000002]
  taus13 = bop + [nan, 1e-3, 0.0]
  for seed, taus in ((21, bop), (22, taus10), (23, taus13)):
    _fused_vs_oracle(oracle_mod, seed, n, 640, 480, synth.LMO_K, 20, 40, taus=taus, dia=dia)
  # float64 delta not representable in float32, both comparison modes
  for f64 in (False, True):
    _fused_vs_oracle(oracle_mod, 24, 8, 640, 480, synth.LMO_K, 20, 40, delta=15.3,
                     delta_f64=f64)


def _bumpy_mesh(seed, n_lat=40, n_lon=80, amp=0.35):
  """Non-convex closed mesh (radial noise on a superellipsoid): self-occlusion,
  folds and near-edge-on slivers for the occlusion test and the spec v5 clamp."""
  from bop_toolkit_amd import synth
  rng = np.random.default_rng(seed)
  pts, faces = synth.superellipsoid(n_lat, n_lon, (50.0, 40.0, 60.0), 0.8)
  pts = pts * (1.0 + amp * rng.uniform(-1.0, 1.0, (len(pts), 1)))
  return pts.astype(np.float32).astype(np.float64), faces


@pytest.mark.parametrize("cull,qorder", [("1", "1"), ("0", "1"), ("1", "0"), ("0", "0"),
                                         ("3", "1")])
def test_fused_vsd_occlusion_cull_exact(oracle_mod, monkeypatch, cull, qorder):
  """k_vsd's occlusion test of far meshlet entries (BOPX_VSD_CULL) and both
  tile entry-queue orders (BOPX_VSD_QORDER: large overlaps first / near first)
  on a non-convex mesh and on an almost flat one (edge-on views: irregular,
  clamped triangles of raster spec v5): bit-exact vs the oracle every way."""
  from bop_toolkit_amd import synth
  monkeypatch.setenv("BOPX_VSD_CULL", cull)
  monkeypatch.setenv("BOPX_VSD_QORDER", qorder)
  out = _fused_vs_oracle(oracle_mod, 41, 24, 640, 480, synth.YCBV_K, 0, 0,
                         mesh=_bumpy_mesh(3), z_range=(500.0, 900.0))
  assert np.ptp(out) > 0.1
  flat = synth.superellipsoid(30, 60, (70.0, 50.0, 0.02), 0.9)
  _fused_vs_oracle(oracle_mod, 42, 24, 640, 480, synth.LMO_K, 0, 0, mesh=flat)


def test_fused_vsd_backface_cull_open_and_flipped(oracle_mod, monkeypatch):
  """The back-face occlusion test (BOPX_VSD_CULL=3) classifies meshlets with
  normal cones of the mesh's orientation; it must stay bit-exact when that
  classification is wrong: an open mesh (the inside of a bowl is visible) and
  the same mesh with every triangle's winding flipped."""
  from bop_toolkit_amd import synth
  monkeypatch.setenv("BOPX_VSD_CULL", "3")
  pts, faces = _bumpy_mesh(5)
  cen = pts[faces].mean(1)
  bowl = faces[cen[:, 2] < 0.3 * cen[:, 2].max()]
  _fused_vs_oracle(oracle_mod, 43, 24, 640, 480, synth.YCBV_K, 0, 0, mesh=(pts, bowl),
                   z_range=(500.0, 900.0))
  _fused_vs_oracle(oracle_mod, 44, 24, 640, 480, synth.YCBV_K, 0, 0,
                   mesh=(pts, np.ascontiguousarray(faces[:, ::-1])), z_range=(500.0, 900.0))


def test_vsd_more_taus_than_one_launch(oracle_mod):
  """The reference takes any number of taus; the kernels take MAX_TAUS per
  launch, so 25 thresholds run in two launches (drop-in with the HIP renderer,
  drop-in with a foreign renderer, batched): bit-exact vs the oracle."""
  import torch
  from bop_toolkit_amd import pose_error as pe, synth
  from bop_toolkit_amd.batch import BatchEvaluator
  from bop_toolkit_amd.renderer import create_renderer
  rng, pts, faces, Rg, tg, Re, te_, K = _scene(31, 3)
  taus = list(np.linspace(0.02, 0.6, 25))
  fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
  ren = create_renderer(640, 480, "hip", mode="depth")
  ren.add_object_arrays(23, pts, faces)

  class Foreign:
    def render_object(self, obj_id, R, t, fx, fy, cx, cy):
      return {"depth": oracle_mod.render_depth(pts, faces, R, t, fx, fy, cx, cy, 640, 480)}

  ev = BatchEvaluator(0)
  ev.add_object(23, pts, faces)
  for i in range(3):
    dg = oracle_mod.render_depth(pts, faces, Rg[i], tg[i], fx, fy, cx, cy, 640, 480)
    de = oracle_mod.render_depth(pts, faces, Re[i], te_[i], fx, fy, cx, cy, 640, 480)
    dt = np.where(dg > 0, dg + 2.0, 0.0).astype(np.float32)
    ref = oracle_mod.vsd_depths(dt, de, dg, fx, fy, cx, cy, 15.0, taus, True, 150.0)
    for r in (ren, Foreign()):
      assert pe.vsd(Re[i], te_[i].reshape(3, 1), Rg[i], tg[i].reshape(3, 1), dt, K, 15.0, taus,
                    True, 150.0, r, 23, "step") == ref
    T = lambda a, dt_=torch.float64: torch.as_tensor(np.asarray(a), dtype=dt_, device=ev.device)
    out = ev.vsd(ev.slots([23]),
                 T(np.concatenate([Re[i].reshape(9), te_[i]])[None]),
                 T(np.concatenate([Rg[i].reshape(9), tg[i]])[None]), T([0], torch.int32),
                 T(dt[None], torch.float32), T([[fx, fy, cx, cy]]), 15.0, taus, T([150.0]))
    assert out.cpu().numpy()[0].tolist() == ref


def test_drop_in_vsd_with_hip_renderer(oracle_mod):
  from bop_toolkit_amd import pose_error as pe, synth
  from bop_toolkit_amd.renderer import create_renderer
  rng, pts, faces, Rg, tg, Re, te_, K = _scene(15, 6)
  ren = create_renderer(640, 480, "hip", mode="depth")
  ren.add_object_arrays(21, pts, faces)
  fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
  taus = list(np.arange(0.05, 0.51, 0.05))
  for i in range(6):
    dg = oracle_mod.render_depth(pts, faces, Rg[i], tg[i], fx, fy, cx, cy, 640, 480)
    dt = np.where(dg > 0, dg + 1.0, 0.0).astype(np.float32)
    e = pe.vsd(Re[i], te_[i].reshape(3, 1), Rg[i], tg[i].reshape(3, 1), dt, K, 15.0, taus, True,
               150.0, ren, 21, "step")
    de = oracle_mod.render_depth(pts, faces, Re[i], te_[i], fx, fy, cx, cy, 640, 480)
    assert e == oracle_mod.vsd_depths(dt, de, dg, fx, fy, cx, cy, 15.0, taus, True, 150.0)
    # est == gt on its own render: VSD = 0
    e0 = pe.vsd(Rg[i], tg[i].reshape(3, 1), Rg[i], tg[i].reshape(3, 1), dt, K, 15.0, taus,
                True, 150.0, ren, 21, "step")
    assert e0 == [0.0] * len(taus)


def test_batch_evaluator_matches_oracle(oracle_mod):
  import torch
  from bop_toolkit_amd import misc, synth
  from bop_toolkit_amd.batch import BatchEvaluator
  rng = np.random.default_rng(21)
  ev = BatchEvaluator(0)
  objs = []
  for o, (nd, cont) in enumerate([(1, False), (4, False), (2, False), (1, True)]):
    pts, faces = synth.superellipsoid(16, 32, (30.0 + 5 * o, 40.0, 50.0 - 5 * o), 0.6 + 0.1 * o)
    info = synth.models_info_entry(pts, nd, cont)
    syms = misc.get_symmetry_transformations(info, 0.01)
    ev.add_object(o, pts, faces, syms, info["diameter"])
    objs.append({"pts": pts, "faces": faces, "syms": misc.symmetries_to_array(syms),
                 "diameter": info["diameter"]})
  n, W, H = 32, 640, 480
  K = synth.LMO_K
  obj = rng.integers(0, 4, n).astype(np.int32)
  Rg, tg = synth.gt_poses(rng, n)
  Re, te_ = synth.perturb(rng, Rg, tg)
  pe = np.concatenate([Re.reshape(n, 9), te_], 1)
  pg = np.concatenate([Rg.reshape(n, 9), tg], 1)
  cam = np.array([[K[0, 0], K[1, 1], K[0, 2], K[1, 2]]])
  dev = ev.device
  t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
  slots = ev.slots(obj)
  fi = np.zeros(n, np.int32)
  # composite test depth of all GT instances in one frame, rendered on the GPU
  frames = ev.render(slots, t(pg, torch.float64), t(fi, torch.int32), t(cam, torch.float64), 1, W,
                     H)
  frames = torch.round(torch.where(frames > 0, frames, torch.full_like(frames, 1500.0)))
  dia = np.array([objs[o]["diameter"] for o in obj])
  Kt = t(np.tile(K.reshape(9), (n, 1)), torch.float64)
  res = ev.bop19(slots, t(pe, torch.float64), t(pg, torch.float64), Kt, t(fi, torch.int32),
                 frames, t(cam, torch.float64), 15.0, np.arange(0.05, 0.51, 0.05),
                 t(dia, torch.float64))
  torch.cuda.synchronize()
  fr = frames.cpu().numpy()
  ref_vsd, ref_mssd, ref_mspd = oracle_mod.bop19_batch(objs, obj, pe, pg, fi, fr, cam, 15.0,
                                                       np.arange(0.05, 0.51, 0.05), dia)
  assert np.array_equal(res["vsd"].cpu().numpy(), ref_vsd)
  np.testing.assert_allclose(res["mssd"].cpu().numpy(), ref_mssd, rtol=0, atol=TOL)
  np.testing.assert_allclose(res["mspd"].cpu().numpy(), ref_mspd, rtol=0, atol=TOL)
  # the composited frame equals the oracle's min-composite of the GT renders
  comp = np.full((H, W), np.inf, np.float32)
  for i in range(n):
    d = oracle_mod.render_depth(objs[obj[i]]["pts"], objs[obj[i]]["faces"], Rg[i], tg[i],
                                K[0, 0], K[1, 1], K[0, 2], K[1, 2], W, H)
    comp = np.where(d > 0, np.minimum(comp, d), comp)
  comp[np.isinf(comp)] = 1500.0
  assert np.array_equal(np.round(comp), fr[0])


def test_sym_pruning_bit_identical(ctx, oracle_mod, monkeypatch):
  """MSSD / MSPD with symmetry pruning (BOPX_SYM_PRUNE, default: units of >= 2
  symmetries) give the same bits as the exhaustive sweep, and match the oracle,
  over discrete sets of 2 .. 64 (one chunk), 65 and 128 (two chunks) and a
  continuous 314-element set, with gross outliers and a pose behind the camera."""
  from bop_toolkit_amd import misc, synth
  rng = np.random.default_rng(77)
  objs = []
  for o, (nd, cont) in enumerate([(2, False), (8, False), (16, False), (64, False), (65, False),
                                  (128, False), (1, True), (2, True)]):
    pts, faces = synth.superellipsoid(12 + 2 * o, 24, (30.0 + 4 * o, 45.0, 55.0 - 3 * o),
                                      0.55 + 0.05 * o)
    pts = pts * (1.0 + 0.2 * rng.uniform(-1.0, 1.0, (len(pts), 1)))  # non-convex
    info = synth.models_info_entry(pts, nd, cont)
    syms = misc.symmetries_to_array(misc.get_symmetry_transformations(info, 0.01))
    ctx.add_object(700 + o, pts, faces)
    ctx.set_symmetries(700 + o, syms)
    objs.append({"pts": pts, "faces": faces, "syms": syms})
  n = 96
  obj = (np.arange(n) % len(objs)).astype(np.int32)
  Rg, tg = synth.gt_poses(rng, n)
  Re, te_ = synth.perturb(rng, Rg, tg, outlier_frac=0.3)
  te_[5, 2] = -50.0  # estimate behind the camera (MSPD: negative / tiny depths)
  pe = np.concatenate([Re.reshape(n, 9), te_], 1)
  pg = np.concatenate([Rg.reshape(n, 9), tg], 1)
  K = np.tile(synth.LMO_K.reshape(9), (n, 1))
  res = {}
  for mode in ("0", "8", "2"):
    monkeypatch.setenv("BOPX_SYM_PRUNE", mode)
    res[mode] = (_batch(ctx, "bopx_mssd_batch", obj + 700, pe, pg),
                 _batch(ctx, "bopx_mspd_batch", obj + 700, pe, pg, K))
  for mode in ("8", "2"):
    assert np.array_equal(res[mode][0], res["0"][0]), "MSSD pruned != exhaustive"
    assert np.array_equal(res[mode][1], res["0"][1]), "MSPD pruned != exhaustive"
  for i in range(0, n, 5):
    o = objs[obj[i]]
    want = oracle_mod.mssd(o["pts"], o["syms"], pe[i], pg[i])
    assert abs(res["8"][0][i] - want) <= TOL * max(1.0, abs(want))
    if i != 5:
      want = oracle_mod.mspd(o["pts"], o["syms"], pe[i], pg[i], K[i])
      assert abs(res["8"][1][i] - want) <= TOL * max(1.0, abs(want))
  for o in range(len(objs)):
    ctx.remove_object(700 + o)


def test_errors_on_bad_input(ctx):
  from bop_toolkit_amd._lib import _d, _i32, ptr
  ids = np.array([12345], np.int32)
  pe = np.zeros(12)
  out = np.empty(1)
  with pytest.raises(KeyError):
    ctx.call("bopx_mssd_batch", 1, ptr(ids, _i32), ptr(pe, _d), ptr(pe, _d), ptr(out, _d))
  ctx.add_object(77, np.zeros((3, 3)), None)
  with pytest.raises(ValueError):  # no symmetry set registered
    ids = np.array([77], np.int32)
    ctx.call("bopx_mssd_batch", 1, ptr(ids, _i32), ptr(pe, _d), ptr(pe, _d), ptr(out, _d))
  # n == 0 is a no-op
  ctx.call("bopx_mssd_batch", 0, ptr(ids, _i32), ptr(pe, _d), ptr(pe, _d), ptr(out, _d))


def _cover_ref(de, dg):
  """Reference formulas of pose_error.cus / cou_bb_proj (pose_error.py:256-330)
  on two depth maps: union, inter, bboxes (x0, y0, x1, y1; empty: -1)."""
  me, mg = de > 0, dg > 0
  row = [float(np.logical_or(me, mg).sum()), float(np.logical_and(me, mg).sum())]
  for m in (me, mg):
    ys, xs = m.nonzero()
    row += [xs.min(), ys.min(), xs.max(), ys.max()] if len(xs) else [2147483647] * 2 + [-1] * 2
  return np.array(row, np.float64)


def test_cover_bit_exact_vs_oracle(oracle_mod):
  """Silhouette mode of k_vsd (cus, cou_bb_proj) vs the oracle raster: exact
  counts and bboxes, including empty / behind-camera / off-screen poses."""
  from bop_toolkit_amd import _lib, pose_error
  from bop_toolkit_amd._lib import _d, _i32, ptr
  n = 24
  rng, pts, faces, Rg, tg, Re, te_, K = _scene(23, n)
  te_[3] = [0.0, 0.0, -300.0]  # behind the camera: empty est mask
  te_[4] = [5000.0, 0.0, 800.0]  # off-screen
  tg[5] = [0.0, 0.0, 70.0]  # very close: guard band
  ctx = _lib.Context(0)
  ctx.add_object(4, pts, faces)
  fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
  ids = np.full(n, 4, np.int32)
  pe = np.concatenate([Re.reshape(n, 9), te_], 1)
  pg = np.concatenate([Rg.reshape(n, 9), tg], 1)
  fi = np.zeros(n, np.int32)
  cam = np.array([[fx, fy, cx, cy]], np.float64)
  out = np.empty((n, 10))
  ctx.call("bopx_cover_batch", n, ptr(ids, _i32), ptr(pe, _d), ptr(pg, _d), ptr(fi, _i32), 1,
           640, 480, ptr(cam, _d), ptr(out, _d))
  for i in range(n):
    de = oracle_mod.render_depth(pts, faces, Re[i], te_[i], fx, fy, cx, cy, 640, 480)
    dg = oracle_mod.render_depth(pts, faces, Rg[i], tg[i], fx, fy, cx, cy, 640, 480)
    ref = _cover_ref(de, dg)
    assert np.array_equal(out[i], ref), (i, out[i], ref)
    # foreign-renderer path on the same maps
    from bop_toolkit_amd._lib import _f
    o2 = np.empty(10)
    ctx.call("bopx_cover_from_depths", 640, 480, ptr(np.ascontiguousarray(de), _f),
             ptr(np.ascontiguousarray(dg), _f), ptr(o2, _d))
    assert np.array_equal(o2, ref), i
    if ref[0] > 0:
      assert pose_error.cus_from_cover(out[i]) == 1.0 - ref[1] / ref[0]
  ctx.close()


def test_drop_in_cus_cou_bb_proj(oracle_mod):
  """pose_error.cus / cou_bb_proj with the HIP renderer and with a foreign
  (oracle) renderer agree with the reference formulas bit for bit."""
  from bop_toolkit_amd import misc, pose_error
  from bop_toolkit_amd.renderer import create_renderer
  rng, pts, faces, Rg, tg, Re, te_, K = _scene(29, 8)
  ren = create_renderer(640, 480, "hip", mode="depth")
  ren.add_object_arrays(6, pts, faces)

  class Foreign:
    def render_object(self, obj_id, R, t, fx, fy, cx, cy):
      return {"depth": oracle_mod.render_depth(pts, faces, R, t, fx, fy, cx, cy, 640, 480)}

  fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
  for i in range(8):
    de = oracle_mod.render_depth(pts, faces, Re[i], te_[i], fx, fy, cx, cy, 640, 480)
    dg = oracle_mod.render_depth(pts, faces, Rg[i], tg[i], fx, fy, cx, cy, 640, 480)
    me, mg = de > 0, dg > 0
    union = float(np.logical_or(me, mg).sum())
    cus_ref = 1.0 - np.logical_and(me, mg).sum() / union if union > 0 else 1.0
    ys, xs = me.nonzero()
    bbe = misc.calc_2d_bbox(xs, ys)
    ys, xs = mg.nonzero()
    bbg = misc.calc_2d_bbox(xs, ys)
    cou_ref = 1.0 - misc.iou(bbe, bbg)
    for r in (ren, Foreign()):
      assert pose_error.cus(Re[i], te_[i], Rg[i], tg[i], K, r, 6) == cus_ref
      assert pose_error.cou_bb_proj(Re[i], te_[i], Rg[i], tg[i], K, r, 6) == cou_ref


def test_fused_vsd_bit_exact_large_meshes(oracle_mod):
  """Objects with > 256 and > 512 meshlets: the launch sizes the per-thread
  meshlet-rectangle registers to 2 and 4 (RPT), both paths bit-exact."""
  from bop_toolkit_amd import synth
  _fused_vs_oracle(oracle_mod, 15, 6, 640, 480, synth.YCBV_K, 100, 150)  # 30k tris: RPT 2
  _fused_vs_oracle(oracle_mod, 16, 6, 640, 480, synth.LMO_K, 150, 200)   # 60k tris: RPT 4


def test_huge_mesh_streamed_rects(oracle_mod):
  """An object beyond the register-resident limit (> 1024 meshlets, here
  110k triangles): k_vsd recomputes the meshlet rectangles per tile and
  rasterises them in rounds of 2048 entries (RPT 0). VSD and the silhouette
  mode stay bit-exact; no size limit is left."""
  from bop_toolkit_amd import _lib, synth
  from bop_toolkit_amd._lib import _d, _i32, ptr
  _fused_vs_oracle(oracle_mod, 19, 4, 640, 480, synth.LMO_K, 220, 250)
  n = 4
  rng, pts, faces, Rg, tg, Re, te_, K = _scene(20, n, n_lat=220, n_lon=250)
  assert len(faces) > 64 * 1024
  ctx = _lib.Context(0)
  ctx.add_object(4, pts, faces)
  fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
  pe = np.concatenate([Re.reshape(n, 9), te_], 1)
  pg = np.concatenate([Rg.reshape(n, 9), tg], 1)
  cam = np.array([[fx, fy, cx, cy]], np.float64)
  out = np.empty((n, 10))
  ctx.call("bopx_cover_batch", n, ptr(np.full(n, 4, np.int32), _i32), ptr(pe, _d), ptr(pg, _d),
           ptr(np.zeros(n, np.int32), _i32), 1, 640, 480, ptr(cam, _d), ptr(out, _d))
  for i in range(n):
    de = oracle_mod.render_depth(pts, faces, Re[i], te_[i], fx, fy, cx, cy, 640, 480)
    dg = oracle_mod.render_depth(pts, faces, Rg[i], tg[i], fx, fy, cx, cy, 640, 480)
    assert np.array_equal(out[i], _cover_ref(de, dg)), i
  ctx.close()


def test_gt_masks_huge_mesh_vs_oracle(oracle_mod):
  """GT-info mode (calc_gt_masks canvas) on an object beyond the register-
  resident limit (RPT 0): silhouette and visible-part masks and counts equal
  the oracle raster + bop19 visibility on the same test depth."""
  from bop_toolkit_amd import _lib
  from bop_toolkit_amd._lib import _d, _f, _i32, _u8, ptr
  n, W, H = 3, 640, 480
  rng, pts, faces, Rg, tg, Re, te_, K = _scene(21, n, n_lat=220, n_lon=250)
  fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
  ctx = _lib.Context(0)
  ctx.add_object(4, pts, faces)
  frames, dgs = [], []
  for i in range(n):
    dg = oracle_mod.render_depth(pts, faces, Rg[i], tg[i], fx, fy, cx, cy, W, H)
    dt = np.where(dg > 0, dg + rng.normal(0, 8.0, dg.shape), 1600.0).astype(np.float32)
    dt[rng.random(dt.shape) < 0.1] = 0.0
    frames.append(np.round(dt).astype(np.float32))
    dgs.append(dg)
  frames = np.stack(frames)
  pg = np.concatenate([Rg.reshape(n, 9), tg], 1)
  cam = np.tile([fx, fy, cx, cy], (n, 1)).astype(np.float64)
  out = np.empty((n, 11))
  masks = np.zeros((n, 2, H, W), np.uint8)
  ctx.call("bopx_gt_info_batch", n, ptr(np.full(n, 4, np.int32), _i32), ptr(pg, _d),
           ptr(np.arange(n, dtype=np.int32), _i32), ptr(frames, _f), n, W, H, ptr(cam, _d), 15.0,
           0, 1, ptr(out, _d), ptr(masks, _u8))
  for i in range(n):
    d_t = oracle_mod.dist_im(frames[i], fx, fy, cx, cy)
    d_g = oracle_mod.dist_im(dgs[i], fx, fy, cx, cy)
    vis = oracle_mod.visib_mask(d_t, d_g, 15.0)
    assert np.array_equal(masks[i, 0] > 0, dgs[i] > 0), i
    assert np.array_equal(masks[i, 1] > 0, vis), i
    assert out[i, 0] == (dgs[i] > 0).sum() and out[i, 1] == vis.sum(), i
  ctx.close()


def test_fused_vsd_bit_exact_large_images(oracle_mod):
  """ITODD-like 1280x960 (delta 5, dataset_params.py) and HOPE-like 1920x1080
  frames: many tiles per tuple, bit-exact."""
  K_itodd = np.array([[2992.0, 0.0, 640.5], [0.0, 2992.0, 480.5], [0.0, 0.0, 1.0]])
  K_hope = np.array([[1390.0, 0.0, 960.0], [0.0, 1390.0, 540.0], [0.0, 0.0, 1.0]])
  _fused_vs_oracle(oracle_mod, 17, 4, 1280, 960, K_itodd, 30, 60, delta=5.0)
  _fused_vs_oracle(oracle_mod, 18, 4, 1920, 1080, K_hope, 30, 60)


def test_launch_order_large_batch(oracle_mod):
  """Batches of >= 1024 tuples run in the object-grouped launch order
  (k_order_by_slot); the same tuples in chunks of 512 keep the identity order.
  Every error type must give identical bits both ways, and match the oracle."""
  import torch
  from bop_toolkit_amd import misc, synth
  from bop_toolkit_amd.batch import BatchEvaluator
  rng = np.random.default_rng(31)
  ev = BatchEvaluator(0)
  objs = []
  for o, (nd, cont) in enumerate([(1, False), (4, False), (8, False), (1, True)]):
    pts, faces = synth.superellipsoid(12, 24, (30.0 + 5 * o, 40.0, 50.0 - 5 * o), 0.6 + 0.1 * o)
    info = synth.models_info_entry(pts, nd, cont)
    syms = misc.get_symmetry_transformations(info, 0.01)
    ev.add_object(o, pts, faces, syms, info["diameter"])
    objs.append({"pts": pts, "faces": faces, "syms": misc.symmetries_to_array(syms),
                 "diameter": info["diameter"]})
  n, per, W, H = 1536, 16, 640, 480
  n_img = n // per
  K = synth.LMO_K
  obj = rng.integers(0, 4, n).astype(np.int32)
  Rg, tg = synth.gt_poses(rng, n)
  Re, te_ = synth.perturb(rng, Rg, tg)
  dev = ev.device
  t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
  pe = t(np.concatenate([Re.reshape(n, 9), te_], 1), torch.float64)
  pg = t(np.concatenate([Rg.reshape(n, 9), tg], 1), torch.float64)
  cam = t(np.tile([K[0, 0], K[1, 1], K[0, 2], K[1, 2]], (n_img, 1)), torch.float64)
  fi = t(np.repeat(np.arange(n_img), per), torch.int32)
  slots = ev.slots(obj)
  frames = ev.render(slots, pg, fi, cam, n_img, W, H)
  frames = torch.round(torch.where(frames > 0, frames, torch.full_like(frames, 1500.0)))
  Kt = t(np.tile(K.reshape(9), (n, 1)), torch.float64)
  dia = t([objs[o]["diameter"] for o in obj], torch.float64)
  taus = np.arange(0.05, 0.51, 0.05)

  def run(lo, hi):
    s = slice(lo, hi)
    r = ev.bop19(slots[s], pe[s], pg[s], Kt[s], fi[s], frames, cam, 15.0, taus, dia[s])
    r["add"] = ev.add(slots[s], pe[s], pg[s])
    r["adi"] = ev.adi(slots[s], pe[s], pg[s])
    r["proj"] = ev.proj(slots[s], pe[s], pg[s], Kt[s])
    r["cover"] = ev.cover(slots[s], pe[s], pg[s], fi[s], cam, W, H)
    r["gt_info"] = ev.gt_info(slots[s], pg[s], fi[s], frames, cam, 15.0)[0]
    return {k: v.cpu().numpy() for k, v in r.items()}

  full = run(0, n)
  parts = [run(lo, lo + 512) for lo in range(0, n, 512)]
  for k in full:
    assert np.array_equal(full[k], np.concatenate([p[k] for p in parts])), k
  sub = np.arange(0, n, 24)
  fr = frames.cpu().numpy()
  ref_vsd, ref_mssd, ref_mspd = oracle_mod.bop19_batch(
      objs, obj[sub], pe.cpu().numpy()[sub], pg.cpu().numpy()[sub], fi.cpu().numpy()[sub], fr,
      cam.cpu().numpy(), 15.0, taus, dia.cpu().numpy()[sub])
  assert np.array_equal(full["vsd"][sub], ref_vsd)
  np.testing.assert_allclose(full["mssd"][sub], ref_mssd, rtol=0, atol=TOL)
  np.testing.assert_allclose(full["mspd"][sub], ref_mspd, rtol=0, atol=TOL)


def test_adi_split_bit_identical(monkeypatch):
  """ADI's point-range split for small batches (k_adi<true> + k_adi_finish,
  per-query minima merged by atomicMin) gives the same double as one workgroup
  per tuple, for every split count, and matches the oracle (cKDTree-pinned)."""
  from bop_toolkit_amd import _lib, synth
  from oracle import oracle
  rng = np.random.default_rng(41)
  c = _lib.Context(0)
  objs = {}
  for oid, (nl, nn) in {1: (3, 5), 2: (20, 40), 3: (50, 60), 4: (30, 100)}.items():
    pts, faces = synth.superellipsoid(nl, nn, tuple(rng.uniform(30, 90, 3)), 0.7)
    c.add_object(oid, pts, faces)
    objs[oid] = pts
  n = 37
  ids = rng.integers(1, 5, n).astype(np.int32)
  Rg, tg = synth.gt_poses(rng, n)
  Re, te = synth.perturb(rng, Rg, tg)
  pe = np.concatenate([Re.reshape(n, 9), te], 1)
  pg = np.concatenate([Rg.reshape(n, 9), tg], 1)
  outs = {}
  # (point ranges, query-chunk classes) per tuple; ("1", "1") = one workgroup
  for split, qsplit in (("1", "1"), ("2", "1"), ("3", "1"), ("7", "1"), ("64", "1"),
                        ("100000", "1"), ("1", "2"), ("3", "5"), ("7", "1000"), ("1", None),
                        (None, None)):
    for var, v in (("BOPX_ADI_SPLIT", split), ("BOPX_ADI_QSPLIT", qsplit)):
      if v is None:
        monkeypatch.delenv(var, raising=False)
      else:
        monkeypatch.setenv(var, v)
    outs[(split, qsplit)] = _batch(c, "bopx_adi_batch", ids, pe, pg)
  for key, o in outs.items():
    assert np.array_equal(o.view(np.uint64), outs[("1", "1")].view(np.uint64)), key
  want = np.array([oracle.adi(objs[int(ids[i])], pe[i], pg[i]) for i in range(n)])
  assert np.max(np.abs(outs[(None, None)] - want) / np.maximum(1.0, np.abs(want))) < 1e-9


def test_auto_backface_cull_all_modes(oracle_mod, monkeypatch):
  """BOPX_VSD_CULL unset: objects of more than 256 meshlets (here 30k
  triangles) take the back-face occlusion test automatically. Silhouette and
  GT-info modes run the same tile loop, so they are checked too: identical to
  the test switched off (BOPX_VSD_CULL=0) and to the oracle raster."""
  from bop_toolkit_amd import _lib
  from bop_toolkit_amd._lib import _d, _f, _i32, _u8, ptr
  n, W, H = 6, 640, 480
  rng, pts, faces, Rg, tg, Re, te_, K = _scene(47, n, n_lat=100, n_lon=150)
  assert len(faces) > 256 * 64
  fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
  pe = np.concatenate([Re.reshape(n, 9), te_], 1)
  pg = np.concatenate([Rg.reshape(n, 9), tg], 1)
  cam = np.tile([fx, fy, cx, cy], (n, 1)).astype(np.float64)
  ids, fi = np.full(n, 4, np.int32), np.arange(n, dtype=np.int32)
  dgs = [oracle_mod.render_depth(pts, faces, Rg[i], tg[i], fx, fy, cx, cy, W, H)
         for i in range(n)]
  frames = np.stack([np.where(d > 0, d + 3.0, 1500.0) for d in dgs]).astype(np.float32)
  res = {}
  for cull in (None, "0"):
    if cull is None:
      monkeypatch.delenv("BOPX_VSD_CULL", raising=False)
    else:
      monkeypatch.setenv("BOPX_VSD_CULL", cull)
    ctx = _lib.Context(0)
    ctx.add_object(4, pts, faces)
    cov = np.empty((n, 10))
    ctx.call("bopx_cover_batch", n, ptr(ids, _i32), ptr(pe, _d), ptr(pg, _d), ptr(fi, _i32), n,
             W, H, ptr(cam, _d), ptr(cov, _d))
    info = np.empty((n, 11))
    masks = np.zeros((n, 2, H, W), np.uint8)
    ctx.call("bopx_gt_info_batch", n, ptr(ids, _i32), ptr(pg, _d), ptr(fi, _i32),
             ptr(frames, _f), n, W, H, ptr(cam, _d), 15.0, 0, 1, ptr(info, _d), ptr(masks, _u8))
    ctx.close()
    res[cull] = (cov, info, masks)
  for a, b in zip(res[None], res["0"]):
    assert np.array_equal(a, b)
  cov, info, masks = res[None]
  for i in range(n):
    de = oracle_mod.render_depth(pts, faces, Re[i], te_[i], fx, fy, cx, cy, W, H)
    assert np.array_equal(cov[i], _cover_ref(de, dgs[i])), i
    assert np.array_equal(masks[i, 0] > 0, dgs[i] > 0), i


def test_drop_in_vsd_return_types(oracle_mod, monkeypatch):
  """pose_error.vsd returns what the reference returns: a list of numpy.float64
  (pose_error.py:90-91) when the visibility union is non-empty, and the Python
  floats [1.0] * len(taus) for an empty union (:75-76), with the HIP renderer
  and with a foreign one. BOPX_RENDERER_ALIAS=vispy makes the reference's
  default create_renderer(W, H, 'vispy', mode='depth') (eval_calc_errors.py:57,
  188-189) a RendererHIP, so the drop-in is import-only."""
  from bop_toolkit_amd import pose_error as pe
  from bop_toolkit_amd.renderer import create_renderer
  from bop_toolkit_amd.renderer_hip import RendererHIP
  rng, pts, faces, Rg, tg, Re, te_, K = _scene(37, 2)
  monkeypatch.setenv("BOPX_RENDERER_ALIAS", "vispy")
  ren = create_renderer(640, 480, "vispy", mode="depth")
  assert isinstance(ren, RendererHIP)
  ren.add_object_arrays(31, pts, faces)
  fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]

  class Foreign:
    def render_object(self, obj_id, R, t, fx, fy, cx, cy):
      return {"depth": oracle_mod.render_depth(pts, faces, R, t, fx, fy, cx, cy, 640, 480)}

  taus = list(np.arange(0.05, 0.51, 0.05))
  many = list(np.linspace(0.02, 0.6, 20))  # two tau chunks
  dg = oracle_mod.render_depth(pts, faces, Rg[0], tg[0], fx, fy, cx, cy, 640, 480)
  dt = np.where(dg > 0, dg + 1.0, 0.0).astype(np.float32)
  behind = np.array([[0.0], [0.0], [-300.0]])
  for r in (ren, Foreign()):
    for tl in (taus, many):
      e = pe.vsd(Re[0], te_[0].reshape(3, 1), Rg[0], tg[0].reshape(3, 1), dt, K, 15.0, tl, True,
                 150.0, r, 31, "step")
      assert len(e) == len(tl) and all(type(x) is np.float64 for x in e), (type(e[0]), r)
      de = oracle_mod.render_depth(pts, faces, Re[0], te_[0], fx, fy, cx, cy, 640, 480)
      assert e == oracle_mod.vsd_depths(dt, de, dg, fx, fy, cx, cy, 15.0, tl, True, 150.0)
      # both poses behind the camera: empty union, plain floats
      e = pe.vsd(Rg[0], behind, Rg[0], behind, dt, K, 15.0, tl, True, 150.0, r, 31, "step")
      assert e == [1.0] * len(tl) and all(type(x) is float for x in e)
  monkeypatch.delenv("BOPX_RENDERER_ALIAS")
  with pytest.raises(NotImplementedError):
    create_renderer(640, 480, "vispy", mode="depth")



def test_set_symmetries_many_matches_one_by_one(golden_errors):
  """bopx_set_symmetries_many (one call for every object, as Models uploads
  the MSSD / MSPD sets) gives the golden MSSD / MSPD, and refuses an unknown
  object or an empty set without changing anything."""
  from bop_toolkit_amd import _lib
  g = golden_errors
  ctx = _lib.Context(0)
  for o in range(4):
    ctx.add_object(200 + o, g["pts_%d" % o], g["faces_%d" % o])
  ctx.set_symmetries_many([200 + o for o in range(4)], [g["syms_%d" % o] for o in range(4)])
  ids = g["obj"] + 200
  for name in ("mssd", "mspd"):
    K = g["K"] if name == "mspd" else None
    out = _batch(ctx, "bopx_%s_batch" % name, ids, g["pose_est"], g["pose_gt"], K)
    np.testing.assert_allclose(out, g["out_" + name], rtol=0, atol=TOL)
  with pytest.raises(KeyError):
    ctx.set_symmetries_many([200, 999], [g["syms_0"], g["syms_1"]])
  with pytest.raises(ValueError):
    ctx.set_symmetries_many([200], [np.zeros((0, 12))])
  out = _batch(ctx, "bopx_mssd_batch", ids, g["pose_est"], g["pose_gt"])
  np.testing.assert_allclose(out, g["out_mssd"], rtol=0, atol=TOL)
  ctx.close()


def test_preload_code_objects():
  """bopx_preload loads the library's code objects on the context's device (a
  second call is a no-op) and needs no registered object."""
  from bop_toolkit_amd import _lib
  ctx = _lib.Context(0)
  assert ctx.preload() == 0
  assert ctx.preload() == 0
  ctx.close()
