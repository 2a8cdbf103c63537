"""inout.load_ply against the reference reader's output on the committed PLY
fixtures (tests/golden/gen_ply.py): same keys, same float64 values, same
errors for non-triangular faces and bad per-face texture coordinates."""
import json
import os

import numpy as np
import pytest

from bop_toolkit_amd import inout

PLY = os.path.join(os.path.dirname(__file__), "golden", "ply")
META = json.load(open(os.path.join(PLY, "expected.json")))
EXP = np.load(os.path.join(PLY, "expected.npz"))


@pytest.mark.parametrize("name", sorted(META))
def test_load_ply_matches_reference(name):
  m = META[name]
  path = os.path.join(PLY, name)
  if "error" in m:
    with pytest.raises(ValueError, match=m["error"]):
      inout.load_ply(path)
    return
  got = inout.load_ply(path)
  assert sorted(got) == m["keys"]
  assert got.get("texture_file") == m["texture_file"]
  for k in m["keys"]:
    if k == "texture_file":
      continue
    want = EXP["%s|%s" % (name, k)]
    assert got[k].dtype == np.float64 and got[k].shape == want.shape, k
    assert np.array_equal(got[k], want), k


def test_save_ply_round_trip(tmp_path):
  rng = np.random.default_rng(0)
  pts = rng.uniform(-1, 1, (20, 3)).astype(np.float32)
  faces = rng.integers(0, 20, (9, 3))
  path = str(tmp_path / "m.ply")
  inout.save_ply(path, pts, faces)
  m = inout.load_ply(path)
  assert np.array_equal(m["pts"], pts.astype(np.float64))
  assert np.array_equal(m["faces"], faces.astype(np.float64))
