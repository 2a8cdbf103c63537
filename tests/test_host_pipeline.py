"""Host plumbing of the caller scripts (no GPU): the batched depth loader, the
per-process file cache shared by the error-type passes, the staged folder
scorer and the tau chunking of the VSD entry points."""
import os
import time

import numpy as np
import pytest

from bop_toolkit_amd import eval_calc_errors as ece
from bop_toolkit_amd import eval_calc_scores as ecs
from bop_toolkit_amd import inout, pose_error


def _png(path, a):
  from PIL import Image
  Image.fromarray(a.astype(np.uint16)).save(path)


def test_load_depths_scales_and_out(tmp_path):
  """Scaled in float32 in place (eval_calc_errors.py:242-243) and written into a
  caller array; a frame of another size raises instead of being written."""
  rng = np.random.default_rng(3)
  frames = [rng.integers(0, 60000, (6, 8)) for _ in range(5)]
  paths = []
  for k, f in enumerate(frames):
    paths.append(str(tmp_path / ("%d.png" % k)))
    _png(paths[-1], f)
  scales = [0.1, 1.0, 0.25, 0.1, 2.0]
  ref = []
  for f, sc in zip(frames, scales):
    d = f.astype(np.float32)
    d *= sc
    ref.append(d)
  got = inout.load_depths(paths, scales=scales)
  assert all(np.array_equal(a, b) and a.dtype == np.float32 for a, b in zip(got, ref))
  out = np.full((5, 6, 8), -1.0, np.float32)
  assert inout.load_depths(paths, scales=scales, out=out) is out
  assert np.array_equal(out, np.stack(ref))
  with pytest.raises(ValueError):
    inout.load_depths(paths, out=np.empty((5, 6, 9), np.float32))


def test_cached_load_rereads_changed_files(tmp_path):
  path = tmp_path / "a.json"
  path.write_text('{"1": [1, 2]}')
  a = ece.cached_load(inout.load_json, str(path), keys_to_int=True)
  assert a == {1: [1, 2]}
  assert ece.cached_load(inout.load_json, str(path), keys_to_int=True) is a  # cached
  assert ece.cached_load(inout.load_json, str(path)) == {"1": [1, 2]}  # other kwargs
  time.sleep(0.01)
  path.write_text('{"1": [3]}')
  os.utime(path, ns=(time.time_ns(), time.time_ns() + 10 ** 7))
  assert ece.cached_load(inout.load_json, str(path), keys_to_int=True) == {1: [3]}


def test_folder_scorer_in_order_without_pool(monkeypatch):
  """One worker: groups scored at submit time, results in submission order;
  close() is idempotent."""
  monkeypatch.setenv("BOPX_SCORE_NATIVE", "0")  # the Python scorer's process-pool mode
  monkeypatch.setattr(ecs, "_score_job", lambda job: [job[0] + ":" + s for s in job[1]])
  fs = ecs.FolderScorer(3, workers=1)
  fs.submit([("a", ["1", "2"])])
  fs.submit([("b", ["1"]), ("c", [])])
  assert fs.results() == [["a:1", "a:2"], ["b:1"], []]
  fs.close()


def test_folder_scorer_threads_in_order(monkeypatch):
  """Native scorer mode: folders on a thread pool, results in submission order."""
  import time
  monkeypatch.setattr(ecs, "_score_job_threaded", lambda job, cache, thr: (
      time.sleep(0.01 * len(job[1])), [job[0] + ":" + s for s in job[1]])[1])
  fs = ecs.FolderScorer(3, workers=3)
  assert fs.tpool is not None
  fs.submit([("a", ["1", "2", "3"])])
  fs.submit([("b", ["1"]), ("c", [])])
  assert fs.results() == [["a:1", "a:2", "a:3"], ["b:1"], []]
  fs.close()


def test_tau_chunks():
  assert pose_error._tau_chunks(0) == []
  assert pose_error._tau_chunks(10) == [(0, 10)]
  assert pose_error._tau_chunks(16) == [(0, 16)]
  assert pose_error._tau_chunks(25) == [(0, 16), (16, 25)]
  assert pose_error._tau_chunks(33) == [(0, 16), (16, 32), (32, 33)]


def test_save_json_per_value_bytes(tmp_path):
  """The per-tau VSD files written from one encoding per record are the bytes
  save_json writes for the per-tau record lists (several GTs with int keys
  ordered numerically, none, inf, int scores)."""
  import random
  rnd = random.Random(1)
  recs = []
  for _ in range(200):
    gids = rnd.sample(range(15), rnd.choice([0, 1, 1, 2, 3, 11]))
    recs.append({"errors": {g: [rnd.choice([rnd.random(), 1.0, 0.0, float("inf"), 1 / 3, 1e-20])
                                for _ in range(4)] for g in gids},
                 "est_id": rnd.randint(0, 5), "im_id": rnd.randint(0, 3000),
                 "obj_id": rnd.randint(1, 30), "score": rnd.choice([rnd.random(), 1, -2.0])})
  paths = [str(tmp_path / ("f%d.json" % k)) for k in range(4)]
  inout.save_json_per_value(paths, recs, 4)
  for k in range(4):
    ref = str(tmp_path / ("r%d.json" % k))
    inout.save_json(ref, [dict(e, errors={g: [v[k]] for g, v in e["errors"].items()})
                          for e in recs])
    assert open(ref).read() == open(paths[k]).read(), k
  inout.save_json_per_value([str(tmp_path / "e.json")], [], 1)
  inout.save_json(str(tmp_path / "re.json"), [])
  assert open(tmp_path / "e.json").read() == open(tmp_path / "re.json").read()


def test_unique_renders_dedupes_bitwise():
  """batch.unique_renders: one render per distinct (object, frame, float64 pose
  bits); estimates equal to a GT share its render."""
  from bop_toolkit_amd.batch import unique_renders
  rng = np.random.default_rng(3)
  g = rng.normal(size=(3, 12))
  e = rng.normal(size=(3, 12))
  e[0] = g[1]
  pe = np.repeat(e, 3, 0)  # every estimate x every GT
  pg = np.tile(g, (3, 1))
  obj = np.zeros(9, np.int32)
  fi = np.zeros(9, np.int32)
  ro, rp, rf, er, gr = unique_renders(obj, pe, pg, fi)
  assert len(ro) == 5  # 3 GT + 2 new estimates
  assert np.array_equal(rp[er], pe) and np.array_equal(rp[gr], pg)
  # another frame or object: separate renders
  fi2 = fi.copy()
  fi2[:3] = 1
  ro2, rp2, rf2, er2, gr2 = unique_renders(obj, pe, pg, fi2)
  assert len(ro2) > len(ro) and np.array_equal(rf2[er2], fi2) and np.array_equal(rf2[gr2], fi2)
  # -0.0 and 0.0 are different bits: kept apart (the raster sees float32 values
  # that are equal, but a render is keyed by what the caller passed)
  pz = pg.copy()
  pz[0, 9] = 0.0
  pz2 = pz.copy()
  pz2[0, 9] = -0.0
  assert len(unique_renders(obj[:1], pz[:1], pz2[:1], fi[:1])[0]) == 2


def test_vectorised_gates_equal_scalar_gate():
  """ece.gates (vectorised, scalar fallback near the threshold) decides every
  tuple as ece.gate does (eval_calc_errors.py:292-339, misc.py:309-331):
  random poses, tuples placed exactly on / next to the thresholds, zero,
  negative, NaN and infinite depths."""
  rng = np.random.default_rng(3)
  n = 4000
  te = rng.normal(0, 300, (n, 3, 1)) + np.array([[0], [0], [900]])
  tg = te + rng.normal(0, 60, (n, 3, 1))
  dia = rng.uniform(50, 250, n)
  # exactly on the distance threshold, and one ulp either side
  for k, f in ((0, 1.0), (1, np.nextafter(1.0, 2.0)), (2, np.nextafter(1.0, 0.0))):
    dv = np.array([[1.0], [2.0], [2.0]]) / 3.0
    tg[k] = te[k] + dv * dia[k] * f
  te[10, 2, 0] = 0.0
  tg[11, 2, 0] = 0.0
  te[12, 2, 0] = -500.0
  te[13, 0, 0] = np.nan
  tg[14, 1, 0] = np.inf
  tg[15] = te[15]
  for et in ("vsd", "cus", "mssd", "add", "adi", "ad", "mspd"):
    want = np.array([ece.gate(et, float(d), a, b) is not None for d, a, b in zip(dia, te, tg)])
    got = ece.gates(et, dia, list(te), list(tg))
    assert np.array_equal(got, want), et
    assert want.any() and (~want).any() or et == "mspd"


def test_save_json_list_bytes(tmp_path):
  """save_json of lists (errors and matches files) is the element-by-element
  text: dicts with nested dicts / lists, NaN / inf, non-dict elements, and
  strings holding the element separator."""
  import json
  cases = [
      [],
      [{"a": 1}],
      [{"scene_id": 1, "im_id": 2, "error": [0.25], "error_norm": [float("nan")], "valid": True},
       {"scene_id": 1, "im_id": 3, "error": -1, "error_norm": -1, "valid": False}],
      [{"errors": {3: [1.0, float("inf")], 1: [0.5]}, "est_id": 0}, {"errors": {}, "est_id": 1}],
      [{"s": "x}, {y"}, {"s": "z"}],
      [{"a": [{"b": 1}, {"c": 2}]}, {"d": 3}],
      [1, {"a": 2}, [3]],
  ]
  for k, c in enumerate(cases):
    path = tmp_path / ("%d.json" % k)
    inout.save_json(str(path), c)
    want = "[\n" + ",\n".join("  " + json.dumps(e, sort_keys=True) for e in c) + "\n]" if c else "[\n]"
    assert path.read_text() == want, k


def _rand_scene(rng, n_im, n_obj, max_ests, max_inst, tie_scores):
  """targets / ests / scene_gt of one scene in the reference's shapes."""
  scene_gt, targets, ests = {}, {}, []
  for im in range(n_im):
    objs = rng.choice(np.arange(1, 30), n_obj, replace=False).tolist()
    gts = []
    for o in objs:
      for _ in range(int(rng.integers(1, max_inst + 1))):
        gts.append({"obj_id": o, "cam_R_m2c": rng.normal(size=(3, 3)),
                    "cam_t_m2c": rng.normal(size=(3, 1))})
    rng.shuffle(gts)
    scene_gt[im] = gts
    for o in objs:
      targets.setdefault(im, {})[o] = {"scene_id": 5, "im_id": im, "obj_id": o,
                                       "inst_count": int(rng.integers(1, max_inst + 1))}
      for _ in range(int(rng.integers(0, max_ests + 1))):
        ests.append({"scene_id": 5, "im_id": im, "obj_id": o,
                     "score": float(rng.integers(0, 3)) if tie_scores else float(rng.random()),
                     "R": rng.normal(size=(3, 3)), "t": rng.normal(size=(3, 1)), "time": -1.0})
  rng.shuffle(ests)
  return targets, ests, scene_gt


def test_scene_arrays_direct_equals_records_then_arrays():
  """The arrays path builds a scene's arrays without record dicts
  (scene_arrays_direct); they equal scene_arrays(scene_records(...)) for every
  n_top rule, ties, missing estimates, and raise the same errors."""
  rng = np.random.default_rng(17)
  for trial in range(60):
    targets, ests, scene_gt = _rand_scene(rng, int(rng.integers(0, 12)), int(rng.integers(1, 5)),
                                          int(rng.integers(0, 4)), int(rng.integers(1, 3)),
                                          trial % 2 == 0)
    _, ests_org = ece._organize([], ests)
    for n_top in (0, -1, 1, 2, 5):
      for skip in (True, False):
        p = {"n_top": n_top, "skip_missing": skip}
        try:
          recs, n_want = ece.scene_records(p, 5, targets, ests_org, scene_gt)
          want = ece.scene_arrays(recs)
        except Exception as e:  # noqa: BLE001
          with pytest.raises(type(e)) as got_e:
            ece.scene_arrays_direct(p, 5, targets, ests_org, scene_gt)
          assert str(got_e.value) == str(e)
          continue
        got, n_got = ece.scene_arrays_direct(p, 5, targets, ests_org, scene_gt)
        assert n_got == n_want
        assert got.keys() == want.keys()
        for k in want:
          assert got[k].dtype == want[k].dtype and got[k].shape == want[k].shape, k
          assert np.array_equal(got[k], want[k]), k
  # an image of the targets without GT annotations: the same KeyError
  targets, ests, scene_gt = _rand_scene(rng, 3, 2, 2, 1, False)
  del scene_gt[1]
  _, ests_org = ece._organize([], ests)
  p = {"n_top": -1, "skip_missing": True}
  with pytest.raises(KeyError):
    ece.scene_records(p, 5, targets, ests_org, scene_gt)
  with pytest.raises(KeyError):
    ece.scene_arrays_direct(p, 5, targets, ests_org, scene_gt)
