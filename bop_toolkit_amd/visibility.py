"""Visible-surface masks from distance images (mirror of
bop_toolkit_lib/visibility.py), evaluated by the gfx950 kernel k_visib.

Bit-exact with the reference: the model and test distances are rounded to
float32 before the difference (visibility.py:31/35) and compared with `delta`
in float32, the legacy NumPy < 1.24 casting of the reference's pinned runtime
(runtime.delta_flags).
"""
from . import runtime


def _estimate_visib_mask(d_test, d_model, delta, visib_mode="bop19"):
  """Mask of the visible object surface (visibility.py:9-42).

  bop18: visible iff d_model - d_test <= delta and both are valid.
  bop19: pixels with missing test depth (d_test == 0) count as visible.
  """
  assert d_test.shape == d_model.shape
  return runtime.visib_mask(d_test, d_model, delta, visib_mode)


def estimate_visib_mask_gt(d_test, d_gt, delta, visib_mode="bop19"):
  """Visible surface of the model in the GT pose (visibility.py:45-55)."""
  return _estimate_visib_mask(d_test, d_gt, delta, visib_mode)


def estimate_visib_mask_est(d_test, d_est, visib_gt, delta, visib_mode="bop19"):
  """Visible surface in the estimated pose, OR-ed with the GT-visible pixels the
  estimate also covers (visibility.py:58-75, eq. 14 of Hodan et al. ECCVW'16)."""
  assert d_test.shape == d_est.shape
  return runtime.visib_mask(d_test, d_est, delta, visib_mode, visib_gt=visib_gt)
