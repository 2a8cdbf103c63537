"""Host helpers of bop_toolkit_amd.misc that the callers use around the GPU
path (misc.py:191-263, 279-306, 353-361): values checked by hand."""
import numpy as np
import pytest

from bop_toolkit_amd import misc


def test_bboxes_and_clip():
  xs, ys = np.array([-3.0, 5.0, 700.0]), np.array([10.0, 500.0, 20.0])
  assert misc.calc_2d_bbox(xs, ys) == [-3.0, 10.0, 703.0, 490.0]
  assert misc.calc_2d_bbox(xs, ys, (640, 480), clip=True) == [0, 10.0, 639, 469]
  assert misc.clip_pt_to_im([-1, 480], (640, 480)) == [0, 479]
  zs = np.array([2.0, -1.0, 4.0])
  assert misc.calc_3d_bbox(xs, ys, zs) == [-3.0, 10.0, -1.0, 703.0, 490.0, 5.0]


def test_iou():
  assert misc.iou([0, 0, 10, 10], [5, 5, 10, 10]) == 25.0 / 175.0
  assert misc.iou([0, 0, 10, 10], [10, 0, 5, 5]) == 0.0  # touching edges
  assert misc.iou([0, 0, 4, 4], [0, 0, 4, 4]) == 1.0


def test_diameter_and_signatures(tmp_path):
  pts = np.array([[0.0, 0, 0], [3, 4, 0], [1, 1, 1]])
  assert misc.calc_pts_diameter(pts) == 5.0 == misc.calc_pts_diameter2(pts)
  # reference misc.py:286 starts from -1.0; calc_pts_diameter2's np.max raises
  assert misc.calc_pts_diameter(np.zeros((0, 3))) == -1.0
  with pytest.raises(ValueError):
    misc.calc_pts_diameter2(np.zeros((0, 3)))
  # chunked evaluation (rows per chunk shrink with N) = brute force
  rng = np.random.default_rng(3)
  big = rng.normal(size=(3000, 3)) * [100.0, 50.0, 20.0]
  d2 = ((big[:, None, :] - big[None, :, :]) ** 2).sum(-1)
  assert misc.calc_pts_diameter(big) == float(np.sqrt(d2.max()))
  assert misc.get_score_signature([0.3], -1) == "th=0.300_min-visib=-1.000"
  assert misc.get_score_signature([5.0, 5.0], 0.1) == "th=5.000-5.000_min-visib=0.100"
  d = tmp_path / "a" / "b"
  misc.ensure_dir(str(d))
  misc.ensure_dir(str(d))
  assert d.is_dir()


def test_delta_flags_follow_legacy_numpy_casting():
  """float32 d_diff <= scalar delta compares in float32 for every scalar type
  under NumPy < 1.24 (the reference's runtime): np.float64(15.3) included."""
  from bop_toolkit_amd import _lib, runtime
  for delta in (15, 15.0, 15.3, np.float64(15.3), np.float32(15.3), np.int64(15), np.int32(5),
                float("inf"), np.float64("nan")):
    assert runtime.delta_flags(delta) == 0, delta
  assert runtime.delta_flags(1e39) == _lib.DELTA_F64
  assert runtime.delta_flags(np.float64(-1e39)) == _lib.DELTA_F64
  # what the float32 comparison means for delta = 15.3 (not representable):
  # 15.3 rounds to 15.300000190734863 in float32, so d_diff = that value passes
  d = np.float32(15.3)
  assert d <= np.float32(np.float64(15.3)) and not float(d) <= 15.3


def test_renderer_alias_is_opt_in(monkeypatch):
  """create_renderer(W, H, 'vispy') (the reference caller's default,
  eval_calc_errors.py:57,188-189) raises unless BOPX_RENDERER_ALIAS names it;
  then it builds the HIP renderer (stubbed here: no GPU on this host)."""
  from bop_toolkit_amd import renderer, renderer_hip

  class Fake:
    def __init__(self, *a):
      self.args = a

  monkeypatch.setattr(renderer_hip, "RendererHIP", Fake)
  monkeypatch.delenv("BOPX_RENDERER_ALIAS", raising=False)
  with pytest.raises(NotImplementedError):
    renderer.create_renderer(640, 480, "vispy", mode="depth")
  with pytest.raises(ValueError):
    renderer.create_renderer(640, 480, "opengl", mode="depth")
  monkeypatch.setenv("BOPX_RENDERER_ALIAS", "cpp, vispy")
  r = renderer.create_renderer(640, 480, "vispy", mode="depth")
  assert isinstance(r, Fake) and r.args[:3] == (640, 480, "depth")
  assert isinstance(renderer.create_renderer(640, 480, "cpp"), Fake)
  with pytest.raises(NotImplementedError):
    renderer.create_renderer(640, 480, "python")


def test_vsd_result_types():
  """The drop-in VSD's return value (pose_error.py:75-91): numpy.float64
  elements for a non-empty union, Python floats [1.0] * n for an empty one."""
  from bop_toolkit_amd.pose_error import _vsd_result
  e = _vsd_result(np.array([0.25, 1.0]), 40.0)
  assert e == [0.25, 1.0] and all(type(x) is np.float64 for x in e)
  e = _vsd_result(np.array([1.0, 1.0, 1.0]), 0.0)
  assert e == [1.0] * 3 and all(type(x) is float for x in e)


def _same_results(a, b):
  assert len(a) == len(b)
  for x, y in zip(a, b):
    assert x.keys() == y.keys()
    for key in ("scene_id", "im_id", "obj_id", "score", "time"):
      assert type(x[key]) is type(y[key])
      assert x[key] == y[key] or (x[key] != x[key] and y[key] != y[key])  # nan == nan
    for key, shape in (("R", (3, 3)), ("t", (3, 1))):
      assert x[key].shape == y[key].shape == shape and x[key].dtype == y[key].dtype
      assert np.array_equal(x[key].view(np.uint64), y[key].view(np.uint64))


def test_bop_results_native_reader_matches_the_line_reader(tmp_path):
  """inout.load_bop_results (native bopx_read_bop_results for the plain form)
  returns the reference reader's values bit for bit (inout.py:221-261: int()
  of the ids, float() of every number), and files outside the plain form go
  through the line reader: the same values, or the reference's error for the
  first bad line."""
  from bop_toolkit_amd import inout
  rng = np.random.default_rng(3)
  nums = ["%.17g", "%.8f", "%.3e", "%r"]
  special = ["5.", ".5", "+1.25", "-0.0", "0", "1e400", "-1e400", "1e-400", "4.9e-324",
             "0.1234567890123456789012345", "123456789012345678901234567890", "1E5", "-7E-3"]
  header = "scene_id,im_id,obj_id,score,R,t,time\n"

  def row(k):
    f = lambda v: nums[k % 4].replace("%r", "%s") % (repr(float(v)) if nums[k % 4] == "%r" else v)
    R = [f(v) for v in rng.normal(size=9)]
    t = [f(v) for v in rng.normal(size=3) * 1000]
    if k % 5 == 0:
      R[k % 9] = special[k % len(special)]
    sep = "\t" if k % 7 == 0 else " "
    ids = ["%d" % (k % 7), " %d " % k if k % 11 == 0 else "%d" % k, "%03d" % (1 + k % 21)]
    return ",".join(ids + [f(rng.random()), sep.join(R), sep.join(t), "-1" if k % 2 else "0.25"])

  rows = [row(k) for k in range(400)]
  p = str(tmp_path / "r.csv")
  for text in (header + "\n".join(rows) + "\n", "\n".join(rows), header, "", header + rows[0]):
    open(p, "w").write(text)
    lines = text.splitlines(keepends=True)
    want = inout._bop_results_lines(lines[1:] if lines and header.strip() in lines[0] else lines)
    assert inout._bop_results_native(p) is not None
    _same_results(inout.load_bop_results(p), want)
  # outside the plain form: the line reader decides (values or its error)
  body = rows[:30]
  cases = {
      "crlf": "\r\n".join(body) + "\r\n",
      "inf_nan": "\n".join(body[:3] + [body[3].replace(body[3].split(",")[4].split()[0], "nan", 1),
                                       body[4].replace(",0.25", ",inf")]),
      "underscore": "\n".join(body[:2] + [body[2].replace(",", ",1_0", 1)]),
      "non_ascii": header.replace("time", "timé") + "\n".join(body),
      "fields": "\n".join(body[:5] + ["1,2,3"] + body[5:]),
      "bad_float": "\n".join(body[:7] + [body[7].replace(".", "x", 1)]),
      "short_R": "\n".join(body[:4] + [",".join(body[4].split(",")[:4] + ["1 2 3"] +
                                               body[4].split(",")[5:])]),
      "blank_line": "\n".join(body[:3] + [""] + body[3:]),
      "vtab": "\n".join(body[:2] + [body[2].replace(" ", "\v", 1)]),
  }
  for name, text in cases.items():
    open(p, "w", newline="").write(text)
    assert inout._bop_results_native(p) is None, name
    with open(p, "r") as f:
      lines = f.readlines()
    try:
      want = inout._bop_results_lines(lines[1:] if lines and header.strip() in lines[0] else lines)
    except Exception as e:  # noqa: BLE001
      with pytest.raises(type(e)) as got:
        inout.load_bop_results(p)
      assert str(got.value) == str(e), name
    else:
      _same_results(inout.load_bop_results(p), want)
  with pytest.raises(OSError):
    inout.load_bop_results(str(tmp_path / "missing.csv"))


def test_gc_paused_nests_and_restores(monkeypatch):
  """inout.gc_paused: the collector is off inside (nested too) and back to its
  previous state after; BOPX_GC_PAUSE=0 leaves it alone."""
  import gc
  from bop_toolkit_amd import inout
  assert gc.isenabled()
  with inout.gc_paused():
    assert not gc.isenabled()
    with inout.gc_paused():
      assert not gc.isenabled()
    assert not gc.isenabled()
  assert gc.isenabled()
  gc.disable()
  try:
    with inout.gc_paused():
      pass
    assert not gc.isenabled()  # was off: stays off
  finally:
    gc.enable()
  monkeypatch.setenv("BOPX_GC_PAUSE", "0")
  with inout.gc_paused():
    assert gc.isenabled()
  assert gc.isenabled()
