"""Host helpers of bop_toolkit_amd.misc that the callers use around the GPU
path (misc.py:191-263, 279-306, 353-361): values checked by hand."""
import numpy as np

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
  assert misc.get_score_signature([0.3], -1) == "th=0.300_min-visib=-1.000"
  assert misc.get_score_signature([5.0, 5.0], 0.1) == "th=5.000-5.000_min-visib=0.100"
  d = tmp_path / "a" / "b"
  misc.ensure_dir(str(d))
  misc.ensure_dir(str(d))
  assert d.is_dir()
