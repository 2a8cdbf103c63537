"""The raster spec against the reference vispy renderer's own
transform chain (tests/golden/raster_chain.npz, captured from
bop_toolkit_lib/renderer_vispy.py by tests/golden/gen_raster_chain.py).

The fixture holds what the reference hands to OpenGL: the u_mvp uniform
(renderer_vispy.py:519-521; _calc_calib_proj :187-232, pose_cv_to_gl :266-269,
view :441-445), near / far from the bbox corners (:447-452), the float32
vertex positions (:372-374), and its linearisation of read-back z-buffers
(:526-536). Here OpenGL's fixed rules are applied to those numbers:
  * a row-major numpy mat4 uploaded to GLSL is read column-major, so the
    shader's gl_Position = u_mvp^T [p; 1] = [p; 1] u_mvp (row vector form);
  * NDC = clip.xyz / clip.w; viewport (0, 0, W, H) (:476): x_win = (x+1) W/2,
    y_win = (y+1) H/2, z_win = (z+1)/2 (default depth range);
  * GL pixel (i, j) samples window (i + 0.5, j + 0.5); the read-back rows are
    flipped (:529), so image row r is GL row H-1-r: image v = H - y_win.
The result must be the spec's mapping: u = fx X/Z + cx, v = fy Y/Z + cy with
(X, Y, Z) = R p + t, i.e. image pixel (c, r) samples (c + 0.5, r + 0.5); the
read-back depth of a surface point is its eye Z. GL's coverage (fill) rule is
the only raster piece this cannot pin.
"""
import os

import numpy as np
import pytest

PATH = os.path.join(os.path.dirname(__file__), "golden", "raster_chain.npz")


@pytest.fixture(scope="module")
def chain():
  return dict(np.load(PATH))


def _cases(g):
  return range(len(g["case_W"]))


def _gl_window(g, i):
  """Window coordinates GL computes for every model vertex in case i."""
  mvp = g["case_u_mvp"][i].astype(np.float32).astype(np.float64)  # uniforms are float32
  p = g["a_position"].astype(np.float64)
  clip = np.concatenate([p, np.ones((len(p), 1))], 1) @ mvp
  ndc = clip[:, :3] / clip[:, 3:4]
  W, H = g["case_W"][i], g["case_H"][i]
  x_win = (ndc[:, 0] + 1.0) * W / 2.0
  y_win = (ndc[:, 1] + 1.0) * H / 2.0
  z_win = (ndc[:, 2] + 1.0) / 2.0
  return x_win, y_win, z_win, clip[:, 3]


def _eye(g, i):
  R = g["case_R"][i].astype(np.float32).astype(np.float64)  # float32 view (:441-442)
  t = g["case_t"][i].astype(np.float32).astype(np.float64)
  return g["a_position"].astype(np.float64) @ R.T + t


def test_vertices_and_bbox_are_the_models(chain):
  g = chain
  pts = g["pts"]
  assert np.array_equal(g["a_position"], pts.astype(np.float32))
  lo, hi = pts.min(0), pts.max(0)
  c = g["bbox_corners"]
  assert c.shape == (8, 3)
  assert np.allclose(c.min(0), lo, atol=1e-9) and np.allclose(c.max(0), hi, atol=1e-9)


def test_near_far_are_bbox_corner_eye_z(chain):
  """Spec: near / far = min / max eye Z of the model's 8 bbox corners (float32
  view matrix, renderer_vispy.py:447-452)."""
  g = chain
  for i in _cases(g):
    R = g["case_R"][i].astype(np.float32).astype(np.float64)
    t = g["case_t"][i].astype(np.float32).astype(np.float64)
    z = g["bbox_corners"] @ R[2] + t[2]
    assert g["case_near"][i] == pytest.approx(z.min(), rel=1e-12)
    assert g["case_far"][i] == pytest.approx(z.max(), rel=1e-12)


def test_gl_window_coordinates_are_the_spec_pixel_mapping(chain):
  """GL's window coordinates of every vertex under the reference's uniforms
  equal the spec's (u, v) with the row flip: u = x_win, v = H - y_win, and
  w_clip = eye Z. An off-by-half-pixel or unflipped convention would miss by
  0.5 px / hundreds of px; the float32 uniforms leave ~1e-5 px."""
  g = chain
  worst = 0.0
  for i in _cases(g):
    fx, fy, cx, cy = g["case_K"][i]
    H = g["case_H"][i]
    x_win, y_win, _, w = _gl_window(g, i)
    X = _eye(g, i)
    assert (X[:, 2] > 0).all()
    u = fx * X[:, 0] / X[:, 2] + cx
    v = fy * X[:, 1] / X[:, 2] + cy
    du, dv = np.abs(x_win - u), np.abs((H - y_win) - v)
    worst = max(worst, du.max(), dv.max())
    np.testing.assert_allclose(w, X[:, 2], rtol=1e-6)
  assert worst < 1e-4, worst  # measured 1.3e-5 px
  # ... and the spec's own float32 arithmetic (raster.h / oracle, DESIGN §4
  # steps 1-2) lands on the same point
  for i in _cases(g):
    fx, fy, cx, cy = (np.float32(v) for v in g["case_K"][i])
    H = g["case_H"][i]
    R = g["case_R"][i].astype(np.float32)
    t = g["case_t"][i].astype(np.float32)
    p = g["a_position"]
    Xs = [((R[k, 0] * p[:, 0] + R[k, 1] * p[:, 1]) + R[k, 2] * p[:, 2]) + t[k] for k in range(3)]
    iz = np.float32(1.0) / Xs[2]
    us = (fx * Xs[0]) * iz + cx
    vs = (fy * Xs[1]) * iz + cy
    x_win, y_win, _, _ = _gl_window(g, i)
    assert np.abs(us - x_win).max() < 1e-3 and np.abs(vs - (H - y_win)).max() < 1e-3


def test_linearised_depth_is_eye_z(chain):
  """_draw_depth's mult / (dep + addi) of the float32 z_win GL stores for a
  vertex gives its eye Z (the spec's depth value) to float32 z-buffer
  precision; z_win = 1 (cleared buffer) is background 0; the ramp runs from
  near (z_win = 0) to far (z_win -> 1)."""
  g = chain
  nv = len(g["a_position"])
  worst = 0.0
  for i in _cases(g):
    W = g["case_W"][i]
    zrow = g["case_zbuf_row"][i][:W]
    drow = g["case_depth_row"][i][:W]
    _, _, z_win, _ = _gl_window(g, i)
    assert np.array_equal(zrow[:nv], z_win.astype(np.float32))  # the probes: vertex depths
    Z = _eye(g, i)[:, 2]
    rel = np.abs(drow[:nv] - Z) / Z
    worst = max(worst, rel.max())
    near, far = g["case_near"][i], g["case_far"][i]
    ramp = drow[nv:W - 3]
    assert np.all(np.diff(ramp) > 0)  # monotone in the z-buffer value
    assert drow[nv] == pytest.approx(near, rel=1e-9)  # z_win = 0 -> near plane
    assert drow[W - 2] == pytest.approx(far, rel=1e-4)  # z_win -> 1 -> far plane
    assert drow[W - 1] == 0.0  # z_win = 1: background
  # float32 window depth (24-bit-like spacing near 1) -> ~1e-6 relative in Z
  assert worst < 1e-6, worst  # measured 1.7e-8
  # reference dtype under NumPy >= 2: float64 depth (NEP 50 promotion of the
  # float32 buffer by the float64 scalars mult / addi); the spec returns float32
  assert str(g["depth_dtype"]) == "float64"
