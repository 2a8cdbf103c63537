"""End-to-end parity of the batched error caller (bop_toolkit_amd.eval_calc_errors)
with the reference's scripts/eval_calc_errors.py, pinned by the JSON files the
reference wrote on the committed synthetic LM-O-layout dataset
(tests/golden/gen_e2e.py).

CPU: tuple enumeration (n_top, score sort, est_id), GT matching, host gates and
their fills, the JSON layout. GPU: the whole caller, every error file compared
with the reference's (VSD bit-identical text; point errors to float64
rounding; RE/TE exact).
"""
import json
import math
import os

import numpy as np
import pytest

from bop_toolkit_amd import dataset_params, eval_calc_errors as ece, inout, misc

E2E = os.path.join(os.path.dirname(__file__), "golden", "e2e")
RUNS = json.load(open(os.path.join(E2E, "runs.json")))


def _params(et, n_top, eval_path="/nonexistent"):
  return ece.parse_args([
      "--error_type", et, "--n_top", str(n_top), "--result_filenames", RUNS["result"],
      "--results_path", os.path.join(E2E, "results"), "--eval_path", eval_path,
      "--datasets_path", os.path.join(E2E, "datasets")])


def _expected(et, n_top, tau=None):
  sign = misc.get_error_signature(et, n_top, vsd_delta=15.0, vsd_tau=tau) if et == "vsd" \
      else misc.get_error_signature(et, n_top)
  path = os.path.join(E2E, "expected", sign, "errors_000002.json")
  with open(path) as f:
    return path, json.load(f)


def _plan(p):
  dp_split = dataset_params.get_split_params(p["datasets_path"], "lmo", "test")
  dp_model = dataset_params.get_model_params(p["datasets_path"], "lmo", "eval")
  targets = inout.load_json(os.path.join(dp_split["base_path"], p["targets_filename"]))
  ests = inout.load_bop_results(os.path.join(p["results_path"], RUNS["result"]))
  t_org, e_org = ece.organize(targets, ests)
  info = inout.load_json(dp_model["models_info_path"], keys_to_int=True)
  scene_gt = inout.load_scene_gt(dp_split["scene_gt_tpath"].format(scene_id=2))
  assert list(t_org) == [2]
  recs, _ = ece.scene_records(p, 2, t_org[2], e_org, scene_gt)
  return recs, info


@pytest.mark.parametrize("et,n_top", [tuple(r) for r in RUNS["runs"]])
def test_enumeration_and_gates(et, n_top):
  p = _params(et, n_top)
  recs, info = _plan(p)
  _, exp = _expected(et, n_top, p["vsd_taus"][0] if et == "vsd" else None)
  assert len(recs) == len(exp)
  for r, e in zip(recs, exp):
    assert (r["im_id"], r["obj_id"], r["est_id"], r["score"]) == \
        (e["im_id"], e["obj_id"], e["est_id"], e["score"])
    assert [str(g) for g, _ in r["gts"]] == sorted(e["errors"], key=int)
    for gt_id, gt in r["gts"]:
      fill = ece.gate(et, info[r["obj_id"]]["diameter"], r["t"], gt["cam_t_m2c"])
      got = e["errors"][str(gt_id)]
      if fill == "vsd_fill":
        assert got == [1.0]
      elif fill is not None:
        assert got == fill and math.isinf(got[0])


def test_json_layout_round_trip(tmp_path):
  """save_json reproduces the reference's files byte for byte."""
  for et, n_top in RUNS["runs"]:
    path, content = _expected(et, n_top, 0.05 if et == "vsd" else None)
    content = json.load(open(path), object_hook=lambda d: {
        (int(k) if k.lstrip("-").isdigit() else k): v for k, v in d.items()})
    out = tmp_path / "x.json"
    inout.save_json(str(out), content)
    assert out.read_text() == open(path).read()


def test_dataset_params_paths():
  dp = dataset_params.get_split_params(os.path.join(E2E, "datasets"), "lmo", "test")
  assert dp["im_size"] == (640, 480) and dp["scene_ids"] == [2]
  assert os.path.exists(dp["depth_tpath"].format(scene_id=2, im_id=0))
  assert os.path.exists(dp["scene_gt_tpath"].format(scene_id=2))
  dm = dataset_params.get_model_params(os.path.join(E2E, "datasets"), "lmo", "eval")
  assert dm["symmetric_obj_ids"] == [10, 11]
  assert all(os.path.exists(dm["model_tpath"].format(obj_id=o)) for o in dm["obj_ids"])


def _load(path):
  with open(path) as f:
    return f.read(), json.loads(open(path).read())


@pytest.mark.gpu
def test_caller_matches_reference(tmp_path):
  for et, n_top in RUNS["runs"]:
    p = _params(et, n_top, str(tmp_path))
    written = ece.run(p, 0)
    exp_root = os.path.join(E2E, "expected")
    assert len(written) == (len(p["vsd_taus"]) if et == "vsd" else 1)
    for path in written:
      rel = os.path.relpath(path, os.path.join(str(tmp_path), "synth_lmo-test"))
      got_txt, got = _load(path)
      exp_txt, exp = _load(os.path.join(exp_root, rel))
      if et in ("vsd", "cus", "re", "te", "rete"):
        assert got_txt == exp_txt, rel  # bit-identical values
        continue
      assert len(got) == len(exp)
      for g, e in zip(got, exp):
        assert {k: v for k, v in g.items() if k != "errors"} == \
            {k: v for k, v in e.items() if k != "errors"}
        assert sorted(g["errors"]) == sorted(e["errors"])
        for k in e["errors"]:
          a, b = np.array(g["errors"][k]), np.array(e["errors"][k])
          assert np.array_equal(np.isinf(a), np.isinf(b))
          np.testing.assert_allclose(a[~np.isinf(a)], b[~np.isinf(b)], rtol=1e-9, atol=1e-9)


def test_models_registry_reused_across_error_types():
  """ece.Models on a kept evaluator (eval_bop19_pose: VSD, MSSD, MSPD in one
  process): one mesh upload per model, symmetry sets attached when an error
  type first needs them, nothing re-uploaded for the next type; a changed
  max_sym_disc_step resets the sets only; objects of other datasets leave."""
  class FakeEv:
    def __init__(self):
      self.objects, self.calls = {}, []

    def add_object(self, obj_id, pts, faces=None, syms=None, diameter=None):
      self.calls.append(("add", obj_id, syms is not None))
      self.objects[obj_id] = {"ns": 0 if syms is None else len(syms)}

    def remove_object(self, obj_id):
      self.calls.append(("remove", obj_id))
      self.objects.pop(obj_id)

    def set_symmetries(self, obj_id, syms):
      self.calls.append(("syms", obj_id))
      self.objects[obj_id]["ns"] = len(syms)

  ev = FakeEv()
  ev.objects[999] = {"ns": 0}  # an object of another dataset
  runs = []
  for et, step in (("vsd", 15), ("mssd", 15), ("mspd", 15), ("mssd", 10), ("vsd", 10)):
    p = _params(et, -1)
    p["max_sym_disc_step"] = step
    dp_model = dataset_params.get_model_params(p["datasets_path"], "lmo", "eval")
    info = inout.load_json(dp_model["models_info_path"], keys_to_int=True)
    ev.calls = []
    ece.Models(ev, p, dp_model, info)
    runs.append(ev.calls)
  ids = sorted(ev.objects)
  assert 999 not in ev.objects and ids
  assert ("remove", 999) in runs[0]
  assert sorted(c[1] for c in runs[0] if c[0] == "add") == ids  # first pass: every mesh, no syms
  assert all(not c[2] for c in runs[0] if c[0] == "add")
  assert sorted(c[1] for c in runs[1]) == ids and all(c[0] == "syms" for c in runs[1])
  assert runs[2] == []  # MSPD: same symmetry key, nothing to do
  assert sorted(c[1] for c in runs[3]) == ids and all(c[0] == "syms" for c in runs[3])
  assert runs[4] == []  # VSD does not need symmetry sets


@pytest.mark.gpu
def test_caller_shared_oom_falls_back_to_fused(tmp_path, monkeypatch):
  """when the shared-render scratch does not fit (forced here with
  BOPX_SHARED_MAX_BYTES=1, read per call), the caller takes the fused kernel
  for the same tuples: the VSD files stay byte-identical to the reference's."""
  from bop_toolkit_amd import _lib
  monkeypatch.setenv("BOPX_SHARED_MAX_BYTES", "1")
  runs = [r for r in RUNS["runs"] if r[0] == "vsd"]
  assert runs
  for et, n_top in runs:
    p = _params(et, n_top, str(tmp_path))
    written = ece.run(p, 0)
    for path in written:
      rel = os.path.relpath(path, os.path.join(str(tmp_path), "synth_lmo-test"))
      assert _load(path)[0] == _load(os.path.join(E2E, "expected", rel))[0], rel
  # and the shared entry itself reports the cap as an OOM
  import torch
  from bop_toolkit_amd.batch import BatchEvaluator
  from bop_toolkit_amd import synth
  ev = BatchEvaluator(0)
  pts, faces = synth.superellipsoid(10, 20, (40.0, 30.0, 50.0), 0.7)
  ev.add_object(1, pts, faces)
  d = ev.device
  pose = torch.tensor([[1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 600.0]], dtype=torch.float64, device=d)
  z = torch.zeros(1, dtype=torch.int32, device=d)
  with pytest.raises(_lib.BopxOOMError):
    ev.vsd_shared(ev.slots([1]), pose, z, z, z, torch.zeros((1, 480, 640), device=d),
                  torch.tensor([[572.0, 573.0, 320.0, 240.0]], dtype=torch.float64, device=d),
                  15.0, [0.05], torch.tensor([100.0], dtype=torch.float64, device=d))


@pytest.mark.gpu
def test_caller_scene_without_estimates_in_a_failing_group(tmp_path):
  """a scene with targets but no estimates shares a depth-decode
  group with a scene that has them, and the group fails (the estimate-free
  scene's frames are of another size, a ValueError). The estimate-free scene
  only releases its slice; the other scene falls back to per-scene decoding.
  The reference never uses the estimate-free scene's depth
  (eval_calc_errors.py:238-243, used per estimate only), so the pass must
  finish: scene 2's files byte-identical to the reference's, scene 3's the
  empty list save_json writes."""
  import shutil
  from PIL import Image
  ds = tmp_path / "datasets"
  shutil.copytree(os.path.join(E2E, "datasets"), str(ds))
  lmo = ds / "lmo"
  s3 = lmo / "test" / "000003"
  shutil.copytree(str(lmo / "test" / "000002"), str(s3))
  for f in sorted((s3 / "depth").iterdir()):
    Image.fromarray(np.full((240, 320), 700, np.uint16)).save(str(f))  # another size
  tp = lmo / "test_targets_bop19.json"
  targets = json.load(open(str(tp)))
  extra = [dict(t, scene_id=3) for t in targets if t["scene_id"] == 2]
  inout.save_json(str(tp), extra + targets)  # scene 3 first: its release comes first
  out = tmp_path / "eval"
  p = ece.parse_args([
      "--error_type", "vsd", "--n_top", "-1", "--result_filenames", RUNS["result"],
      "--results_path", os.path.join(E2E, "results"), "--eval_path", str(out),
      "--datasets_path", str(ds)])
  written = ece.run(p, 0)
  empty = tmp_path / "empty.json"
  inout.save_json(str(empty), [])
  n2 = 0
  for path in written:
    rel = os.path.relpath(path, os.path.join(str(out), "synth_lmo-test"))
    if rel.endswith("errors_000003.json"):
      assert _load(path)[0] == _load(str(empty))[0], rel
      continue
    n2 += 1
    assert _load(path)[0] == _load(os.path.join(E2E, "expected", rel))[0], rel
  assert n2 == len(p["vsd_taus"])
