"""Native scorer (include/bopx_score.h, bop_toolkit_amd/csrc/score.cpp): the
matches_*.json / scores_*.json of every setting byte-identical to the Python
scorer (which tests/test_scores.py pins to the reference scripts' files), on
the reference's own golden errors files and on randomised folders with
multi-instance images, ties, n_top, visibility thresholds, int and float
values, NaN / infinite errors, rete-style two-element errors and invalid GTs.
Host-only: runs on the CPU."""
import ctypes
import json
import math
import os
import random
import shutil
import struct

import numpy as np
import pytest

from bop_toolkit_amd import eval_calc_scores as ecs
from bop_toolkit_amd import inout, misc

E2E = os.path.join(os.path.dirname(__file__), "golden", "e2e")
RUNS = json.load(open(os.path.join(E2E, "runs.json")))
NAME = os.path.splitext(RUNS["result"])[0]


def _read(path):
  with open(path) as f:
    return f.read()


def _both(p, folder, ths, tmp_path):
  """Scores + files of the native and the Python scorer for settings ths."""
  import copy
  sps = []
  et = os.path.basename(folder).split("_")[0].split("=")[1]
  for th in ths:
    sp = copy.deepcopy(p)
    sp["correct_th"][et] = list(th)
    sps.append(sp)
  nat = ecs.score_error_dir_native(sps, folder, do_print=False)
  assert nat is not None, "the native scorer declined the inputs"
  files = {}
  for (sc, sign) in nat:
    for kind in ("matches", "scores"):
      fn = os.path.join(p["eval_path"], folder, "{}_{}.json".format(kind, sign))
      files[fn] = _read(fn)
      os.remove(fn)
  for sp, (sc, sign) in zip(sps, nat):
    want, wsign = ecs.score_error_dir(sp, folder, do_print=False)
    assert wsign == sign
    assert json.dumps(want, sort_keys=True) == json.dumps(sc, sort_keys=True)
  for fn, text in files.items():
    assert _read(fn) == text, fn
  return nat


def test_float_repr_matches_python():
  lib = inout._io_lib()
  lib.bopx_py_float_repr.argtypes = [ctypes.c_double, ctypes.c_char_p]
  buf = ctypes.create_string_buffer(64)
  rnd = random.Random(5)
  vals = [0.0, -0.0, 1.0, 0.1, 1e16, 1e15, 9999999999999998.0, 1e-4, 1e-5, 5e-324, 1e22,
          1.7976931348623157e308, float("nan"), float("inf"), float("-inf"), 0.30000000000000004]
  for _ in range(20000):
    vals.append(struct.unpack("d", struct.pack("Q", rnd.getrandbits(64)))[0])
    vals.append(rnd.random() * 10 ** rnd.randint(-8, 20))
    vals.append(round(rnd.random(), rnd.randint(0, 17)))
  for v in vals:
    lib.bopx_py_float_repr(v, buf)
    assert buf.value.decode() == inout._json_float(v), repr(v)


@pytest.mark.parametrize("sign,extra", [tuple(r) for r in RUNS["score_runs"]])
def test_native_equals_python_on_golden_errors(tmp_path, sign, extra):
  ev = tmp_path / "eval"
  for root, _, files in os.walk(os.path.join(E2E, "expected")):
    for fn in files:
      if fn.startswith("errors_"):
        rel = os.path.relpath(os.path.join(root, fn), os.path.join(E2E, "expected"))
        dst = ev / NAME / rel
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy(os.path.join(root, fn), dst)
  p = ecs.parse_args(["--error_dir_paths", os.path.join(NAME, sign), "--eval_path", str(ev),
                      "--datasets_path", os.path.join(E2E, "datasets")] + extra)
  et = sign.split("_")[0].split("=")[1]
  base = p["correct_th"][et]
  nat = _both(p, os.path.join(NAME, sign), [base, [t * 0.5 for t in base], [t * 2.0 for t in base]],
              tmp_path)
  # ... and the reference's own files for the setting it ran
  _, ssign = nat[0]
  # (the Python scorer is pinned to them in tests/test_scores.py)
  assert ssign == misc.get_score_signature(base, p["visib_gt_min"])


def _random_dataset(root, seed, n_scenes=3, n_im=25, ints=False, two=False):
  """A small BOP-layout GT side + one errors folder (random errors)."""
  rng = np.random.default_rng(seed)
  ds = os.path.join(root, "datasets", "ycbv")
  os.makedirs(os.path.join(ds, "models_eval"))
  info = {str(o): {"diameter": float(rng.uniform(50, 200))} for o in range(1, 22)}
  with open(os.path.join(ds, "models_eval", "models_info.json"), "w") as f:
    json.dump(info, f)
  targets = []
  errs_by_scene = {}
  for s in range(48, 48 + n_scenes):
    sdir = os.path.join(ds, "test", "%06d" % s)
    os.makedirs(sdir)
    gts, gti, se = {}, {}, []
    for im in range(n_im):
      objs = rng.integers(1, 6, int(rng.integers(1, 6)))
      gts[str(im)] = [{"cam_R_m2c": [1, 0, 0, 0, 1, 0, 0, 0, 1], "cam_t_m2c": [0, 0, 1],
                       "obj_id": int(o)} for o in objs]
      gti[str(im)] = [{"visib_fract": float(np.round(rng.random(), 1))} for _ in objs]
      for o in sorted(set(objs.tolist())):
        cnt = int((objs == o).sum())
        if rng.random() < 0.9:
          targets.append({"im_id": im, "inst_count": cnt, "obj_id": o, "scene_id": s})
        gt_ids = [g for g in range(len(objs)) if objs[g] == o]
        for est in range(int(rng.integers(0, 4))):
          def val():
            r = rng.random()
            if r < 0.03:
              return float("nan")
            if r < 0.06:
              return float("inf")
            v = float(np.round(rng.random() * 0.8, 2))
            return int(v * 10) if ints and r < 0.3 else v
          errors = {g: ([val(), val()] if two else [val()]) for g in rng.permutation(gt_ids)}
          score = float(rng.integers(0, 4)) if rng.random() < 0.5 else float(rng.random())
          se.append({"errors": {int(g): v for g, v in errors.items()}, "est_id": est,
                     "im_id": im, "obj_id": o, "score": score})
      # an estimate of an object the image does not show (ignored by matching)
      se.append({"errors": {}, "est_id": 9, "im_id": im, "obj_id": 21, "score": 0.5})
    for fn, c in (("scene_gt.json", gts), ("scene_gt_info.json", gti)):
      with open(os.path.join(sdir, fn), "w") as f:
        json.dump(c, f)
    errs_by_scene[s] = se
  with open(os.path.join(ds, "test_targets_bop19.json"), "w") as f:
    json.dump(targets, f)
  return errs_by_scene


@pytest.mark.parametrize("seed", range(8))
def test_native_equals_python_random(tmp_path, seed):
  et = ["vsd", "mssd", "mspd", "rete"][seed % 4]
  ints = seed % 3 == 0
  errs = _random_dataset(str(tmp_path), seed, ints=ints, two=et == "rete")
  n_top = [-1, 0, 1, 2][seed % 4]
  sign = "error={}_ntop={}".format(et, n_top)
  folder = os.path.join("m_ycbv-test", sign)
  for s, se in errs.items():
    path = os.path.join(str(tmp_path), "eval", folder, "errors_%06d.json" % s)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    inout.save_json(path, se)
  visib = ["-1", "0.3"][seed % 2]
  p = ecs.parse_args(["--error_dir_paths", folder, "--eval_path", str(tmp_path / "eval"),
                      "--datasets_path", str(tmp_path / "datasets"), "--visib_gt_min", visib])
  ths = {"vsd": [[0.3], [0.05], [0.5]], "mssd": [[0.2], [0.4]], "mspd": [[10.0], [25.0]],
         "rete": [[0.5, 0.4], [0.2, 0.7]]}[et]
  if et == "mspd":  # width-normalised values of any size
    for s, se in errs.items():
      for e in se:
        for g in e["errors"]:
          e["errors"][g] = [v * 40 if isinstance(v, float) and math.isfinite(v) else v
                            for v in e["errors"][g]]
      inout.save_json(os.path.join(str(tmp_path), "eval", folder, "errors_%06d.json" % s), se)
  _both(p, folder, ths, tmp_path)


def test_native_declines_what_python_handles(tmp_path):
  """NaN scores and a missing errors file go to the Python path (None)."""
  errs = _random_dataset(str(tmp_path), 3, n_scenes=1, n_im=4)
  folder = os.path.join("m_ycbv-test", "error=vsd_ntop=-1")
  s, se = next(iter(errs.items()))
  p = ecs.parse_args(["--error_dir_paths", folder, "--eval_path", str(tmp_path / "eval"),
                      "--datasets_path", str(tmp_path / "datasets")])
  assert ecs.score_error_dir_native([p], folder) is None  # no errors file
  se[0]["score"] = float("nan")
  path = os.path.join(str(tmp_path), "eval", folder, "errors_%06d.json" % s)
  os.makedirs(os.path.dirname(path), exist_ok=True)
  inout.save_json(path, se)
  assert ecs.score_error_dir_native([p], folder) is None


@pytest.mark.parametrize("n_values", [1, 10])
def test_native_errors_writer_bytes(tmp_path, n_values):
  """bopx_write_errors = save_json_per_value / save_json of the record dicts
  (several GTs per record, none, fills 1.0 / inf, tiny and large values)."""
  rnd = random.Random(n_values)
  recs, im, ob, est, sc, off, gt, vals = [], [], [], [], [], [0], [], []
  for _ in range(300):
    gids = sorted(rnd.sample(range(15), rnd.choice([0, 1, 1, 2, 3, 11])))
    errors = {g: [rnd.choice([rnd.random(), 1.0, 0.0, float("inf"), 1 / 3, 1e-20, 123456.75,
                              rnd.random() * 1e17]) for _ in range(n_values)] for g in gids}
    r = {"errors": errors, "est_id": rnd.randint(0, 5), "im_id": rnd.randint(0, 3000),
         "obj_id": rnd.randint(1, 21), "score": rnd.choice([rnd.random(), 1.0, 0.5e-7])}
    recs.append(r)
    im.append(r["im_id"]), ob.append(r["obj_id"]), est.append(r["est_id"]), sc.append(r["score"])
    gt += gids
    vals += [errors[g] for g in gids]
    off.append(len(gt))
  want = [str(tmp_path / ("w%d.json" % k)) for k in range(n_values)]
  got = [str(tmp_path / ("g%d.json" % k)) for k in range(n_values)]
  if n_values == 1:
    inout.save_json(want[0], recs)
  else:
    inout.save_json_per_value(want, recs, n_values)
  inout.save_errors_arrays(got, im, ob, est, sc, off, gt,
                           np.array(vals, np.float64).reshape(len(gt), n_values))
  for w, g in zip(want, got):
    assert _read(w) == _read(g)
  inout.save_errors_arrays([got[0]], [], [], [], [], [0], [], np.zeros((0, 1)))
  assert _read(got[0]) == "[\n]"
