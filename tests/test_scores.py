"""Scoring parity: pose matching, recall and the BOP19
average recalls against the files the reference's eval_calc_scores.py and
eval_bop19_pose.py wrote on the golden dataset (tests/golden/gen_e2e.py).
Scores are host bookkeeping, so the CPU tests start from the reference's own
errors_*.json; the GPU test runs the whole BOP19 evaluation (errors on the GPU).
"""
import json
import os
import shutil

import numpy as np
import pytest

from bop_toolkit_amd import eval_bop19_pose as e19
from bop_toolkit_amd import eval_calc_scores as ecs
from bop_toolkit_amd import inout, pose_matching, score

E2E = os.path.join(os.path.dirname(__file__), "golden", "e2e")
RUNS = json.load(open(os.path.join(E2E, "runs.json")))
NAME = os.path.splitext(RUNS["result"])[0]


def _eval_dir_with_errors(tmp_path):
  ev = tmp_path / "eval"
  for root, _, files in os.walk(os.path.join(E2E, "expected")):
    for fn in files:
      if fn.startswith("errors_"):
        rel = os.path.relpath(os.path.join(root, fn), os.path.join(E2E, "expected"))
        dst = ev / NAME / rel
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy(os.path.join(root, fn), dst)
  return ev


def _same_text(a, b):
  assert open(a).read() == open(b).read(), (a, b)


@pytest.mark.parametrize("sign,extra", [tuple(r) for r in RUNS["score_runs"]])
def test_calc_scores_matches_reference(tmp_path, sign, extra):
  ev = _eval_dir_with_errors(tmp_path)
  p = ecs.parse_args(["--error_dir_paths", os.path.join(NAME, sign), "--eval_path", str(ev),
                      "--datasets_path", os.path.join(E2E, "datasets")] + extra)
  _, ssign = ecs.score_error_dir(p, os.path.join(NAME, sign), do_print=False)
  for kind in ("scores", "matches"):
    fn = "{}_{}.json".format(kind, ssign)
    _same_text(ev / NAME / sign / fn, os.path.join(E2E, "expected", sign, fn))


def test_bop19_scores_from_reference_errors(tmp_path, monkeypatch):
  ev = _eval_dir_with_errors(tmp_path)
  monkeypatch.setenv("BOP_PATH", os.path.join(E2E, "datasets"))
  p = e19.parse_args(["--result_filenames", RUNS["result"], "--results_path",
                      os.path.join(E2E, "results"), "--eval_path", str(ev)])
  e19.evaluate(p, calc_errors=False)
  exp = os.path.join(E2E, "expected_bop19")
  n = 0
  for root, _, files in os.walk(exp):
    for fn in files:
      rel = os.path.relpath(os.path.join(root, fn), exp)
      _same_text(ev / NAME / rel, os.path.join(root, fn))
      n += 1
  assert n == 1 + 10 * 10 + 10 + 10  # final + VSD (10 tau x 10 th) + MSSD + MSPD


def test_match_poses_greedy_rules():
  errs = [{"est_id": 0, "score": 0.9, "errors": {0: [0.2], 1: [0.1]}},
          {"est_id": 1, "score": 0.9, "errors": {0: [0.05], 1: [0.3]}},  # tie: stable order
          {"est_id": 2, "score": 0.1, "errors": {0: [0.01], 1: [0.01]}}]
  m = pose_matching.match_poses(errs, [0.25])
  assert [(x["est_id"], x["gt_id"]) for x in m] == [(0, 1), (1, 0)]
  assert m[0]["error_norm"] == [0.1 / 0.25]
  assert pose_matching.match_poses(errs, [0.25], max_ests_count=1)[0]["gt_id"] == 1
  assert pose_matching.match_poses(errs, [0.25], gt_valid_mask=[True, False])[0]["gt_id"] == 0
  # rete-style: every element must be lowest so far
  e2 = [{"est_id": 0, "score": 1.0, "errors": {0: [1.0, 4.0], 1: [2.0, 3.0]}}]
  assert pose_matching.match_poses(e2, [5.0, 5.0])[0]["gt_id"] == 0


def _match_scene_plain(scene_gt, valid, errs, th, n_top):
  """Unoptimised restatement of pose_matching.py:93-160 (flat list, fresh sort
  and the all-elements rule for every group) to check the scalar fast path."""
  out = []
  for im_id, im_gts in scene_gt.items():
    recs = [[-1, -1, -1, -1] for _ in im_gts]  # est_id, score, error, error_norm
    for obj_id in set(g["obj_id"] for g in im_gts):
      group = [e for e in errs if e["im_id"] == im_id and e["obj_id"] == obj_id]
      for m in pose_matching.match_poses(group, th, n_top, valid[im_id]):
        recs[m["gt_id"]] = [m["est_id"], m["score"], m["error"], m["error_norm"]]
    out += recs
  return out


@pytest.mark.parametrize("seed", range(6))
def test_match_scene_fast_path_equals_plain(seed):
  rng = np.random.default_rng(seed)
  scene_gt, valid, errs = {}, {}, []
  for im in range(30):
    objs = rng.integers(1, 5, int(rng.integers(1, 6)))
    scene_gt[im] = [{"obj_id": int(o)} for o in objs]
    valid[im] = [bool(v) for v in rng.random(len(objs)) < 0.8]
    for o in set(objs.tolist()):
      gts = [g for g in range(len(objs)) if objs[g] == o]
      for k in range(int(rng.integers(0, 4))):
        vals = np.round(rng.random(len(gts)), 1)  # ties in errors and scores
        errs.append({"im_id": im, "obj_id": o, "est_id": k, "score": float(rng.integers(0, 3)),
                     "errors": {g: [float(v)] for g, v in zip(gts, vals)}})
  for n_top in (-1, 0, 1, 2):
    for th in ([0.35], [0.75]):
      fast = pose_matching.match_poses_scene(1, scene_gt, valid, errs, th, n_top)
      grouped = pose_matching.match_poses_scene(
          1, scene_gt, valid, pose_matching.group_scene_errs(errs), th, n_top)
      plain = _match_scene_plain(scene_gt, valid, errs, th, n_top)
      got = [[r["est_id"], r["score"], r["error"], r["error_norm"]] for r in fast]
      assert got == plain
      assert grouped == fast


def test_save_json_layout(tmp_path):
  """Fast writer = the reference's per-element json.dumps(sort_keys=True)."""
  content = [{"b": [float("inf"), 0.1 + 0.2, -0.0], "a": {3: True, 10: None}, "s": "x\u00e9"},
             {"errors": {12: [1e-300], 0: [0.5]}, "score": 0.25}]
  path = tmp_path / "x.json"
  inout.save_json(str(path), content)
  want = "[\n" + ",\n".join("  " + json.dumps(e, sort_keys=True) for e in content) + "\n]"
  assert path.read_text() == want
  for empty, text in (([], "[\n]"), ({}, "{\n}")):
    inout.save_json(str(path), empty)
    assert path.read_text() == text
  inout.save_json(str(path), {2: [1, 2], 1: "a"})
  assert path.read_text() == '{\n  "1": "a",\n  "2": [1, 2]\n}'


def test_ap_and_recall():
  assert score.calc_recall(0, 0) == 0.0
  assert score.calc_recall(3, 4) == 0.75
  # envelope of (0.5, 1.0), (1.0, 0.5): 0.5 * 1.0 + 0.5 * 0.5
  assert score.calc_ap([1.0, 0.5], [0.5, 1.0]) == 0.75


def test_average_time_rules():
  assert e19.average_time_per_image([{"scene_id": 1, "im_id": 0, "time": -1.0}]) == -1.0
  with pytest.raises(ValueError):
    e19.average_time_per_image([{"scene_id": 1, "im_id": 0, "time": 0.5},
                                {"scene_id": 1, "im_id": 0, "time": 0.7}])


@pytest.mark.gpu
def test_bop19_end_to_end(tmp_path, monkeypatch):
  monkeypatch.setenv("BOP_PATH", os.path.join(E2E, "datasets"))
  ev = tmp_path / "eval"
  p = e19.parse_args(["--result_filenames", RUNS["result"], "--results_path",
                      os.path.join(E2E, "results"), "--eval_path", str(ev)])
  e19.evaluate(p, 0)
  exp = os.path.join(E2E, "expected_bop19")
  for root, _, files in os.walk(exp):
    for fn in files:
      rel = os.path.relpath(os.path.join(root, fn), exp)
      _same_text(ev / NAME / rel, os.path.join(root, fn))
