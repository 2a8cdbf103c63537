"""GT-side parity: bop_toolkit_amd.gt_side against the
scene_gt_info.json and the masks the reference's scripts/calc_gt_info.py and
scripts/calc_gt_masks.py wrote on the golden dataset (tests/golden/gen_e2e.py;
the reference renderer slot was filled by the CPU raster twin, so raster spec
v4 holds on both sides)."""
import os
import shutil

import numpy as np
import pytest

from bop_toolkit_amd import gt_side

E2E = os.path.join(os.path.dirname(__file__), "golden", "e2e")
EXP = os.path.join(E2E, "expected_gt")


def test_info_row_rules():
  row = np.array([100, 0, 5, 6, 9, 9, 2147483647, 2147483647, -1, -1, 40], np.float64)
  e = gt_side.info_from_row(row)
  assert e == {"px_count_all": 100, "px_count_valid": 40, "px_count_visib": 0,
               "visib_fract": 0.0, "bbox_obj": [-1, -1, -1, -1], "bbox_visib": [-1, -1, -1, -1]}
  row[1] = 30
  row[6:10] = [6, 7, 8, 9]
  e = gt_side.info_from_row(row)
  assert e["visib_fract"] == 0.3 and e["bbox_obj"] == [5, 6, 4, 3]
  assert e["bbox_visib"] == [6, 7, 2, 2]
  assert gt_side.info_from_row(np.zeros(11))["visib_fract"] == 0.0


def _dataset_copy(tmp_path):
  root = tmp_path / "ds"
  shutil.copytree(os.path.join(E2E, "datasets"), root)
  split = root / "lmo" / "test"
  shutil.copytree(split / "000002", split / "000000")
  shutil.copytree(root / "lmo" / "models_eval", root / "lmo" / "models")
  return root


def _params(root, scene):
  return {"dataset": "lmo", "dataset_split": "test", "dataset_split_type": None, "delta": 15,
          "renderer_type": "hip", "datasets_path": str(root), "scene_ids": [scene]}


@pytest.mark.gpu
def test_calc_gt_info_matches_reference(tmp_path):
  root = _dataset_copy(tmp_path)
  (path,) = gt_side.calc_gt_info(_params(root, 2))
  assert open(path).read() == open(os.path.join(EXP, "scene_gt_info_000002.json")).read()


@pytest.mark.gpu
def test_calc_gt_masks_matches_reference(tmp_path):
  from PIL import Image
  root = _dataset_copy(tmp_path)
  written = gt_side.calc_gt_masks(_params(root, 0))
  exp = np.load(os.path.join(EXP, "masks_scene0.npz"))
  assert len(written) == len(exp.files)
  for path in written:
    kind = os.path.basename(os.path.dirname(path))
    key = "%s_%s" % (kind, os.path.splitext(os.path.basename(path))[0])
    m = np.asarray(Image.open(path))
    assert set(np.unique(m)) <= {0, 255}
    assert np.array_equal(np.packbits(m > 0), exp[key]), key


def test_save_scene_gt_info_bytes(tmp_path):
  """The direct writer gives save_json's bytes for the info_from_row dicts:
  visible and invisible instances, empty images, zero silhouettes, fractions
  that need 17 digits, negative box corners."""
  from bop_toolkit_amd import gt_side, inout
  rng = np.random.default_rng(11)
  rows = {}
  for im in (0, 3, 12, 7, 100, 2):
    n = int(rng.integers(0, 5))
    r = np.zeros((n, 11))
    r[:, 0] = rng.integers(0, 300000, n)
    r[:, 1] = np.minimum(r[:, 0], rng.integers(0, 300000, n))
    r[:, 10] = rng.integers(0, 300000, n)
    r[:, 2:10] = rng.integers(-700, 2000, (n, 8))
    if n:
      r[0, 1] = 0
    if n > 1:
      r[1, 0] = r[1, 1] = 0
    rows[im] = list(r)
  a, b = tmp_path / "a.json", tmp_path / "b.json"
  inout.save_json(str(a), {im: [gt_side.info_from_row(x) for x in lst] for im, lst in rows.items()})
  gt_side.save_scene_gt_info(str(b), rows)
  assert a.read_bytes() == b.read_bytes()
  inout.save_json(str(a), {})
  gt_side.save_scene_gt_info(str(b), {})
  assert a.read_bytes() == b.read_bytes()
