"""Batched counterpart of scripts/eval_calc_errors.py.

Same parameters, command line, tuple enumeration and output files as the
reference script (eval_calc_errors.py:23-136 parameters, :137-424 loop):

  * estimates per (scene, image, object) sorted by score, descending and
    stable, est_id = index in the per-(image, object) list; the n_top rule
    (0 = all, -1 = target inst_count, N = top N) (:247-277);
  * errors against every GT instance of the same object in the image (:288-290);
  * the host gates and their fills: VSD/CUS 1.0 when the projected bounding
    spheres do not overlap, AD*/MSSD inf when the centres are a diameter or
    more apart; MSPD ungated (:296-339);
  * errors_{scene:06d}.json per error signature, VSD split per tau (:380-415),
    written with inout.save_json's one-element-per-line layout.

What differs is the evaluation: instead of one pose_error call per tuple, the
gated-in tuples of a scene go to the GPU as one batch per error type
(bop_toolkit_amd.batch: k_vsd fuses both renders, the three distance images,
both visibility masks and the per-tau costs; MSSD/MSPD/ADD/ADI/PROJ are one
launch each). RE/TE are 3x3 host arithmetic, kept on the host as in the
reference. The HIP rasteriser replaces the OpenGL renderer, whatever
--renderer_type says.

    python -m bop_toolkit_amd.eval_calc_errors --error_type vsd --result_filenames ...
"""
import argparse
import copy
import os
import threading
import time

import numpy as np

from . import dataset_params, depth_gpu, inout, misc, pose_error

DEFAULTS = {
    "n_top": 1,
    "error_type": "vsd",
    "vsd_deltas": {"hb": 15, "icbin": 15, "icmi": 15, "itodd": 5, "lm": 15, "lmo": 15,
                   "ruapc": 15, "tless": 15, "tudl": 15, "tyol": 15, "ycbv": 15, "hope": 15},
    "vsd_taus": list(np.arange(0.05, 0.51, 0.05)),
    "vsd_normalized_by_diameter": True,
    "max_sym_disc_step": 0.01,
    "skip_missing": True,
    "renderer_type": "vispy",
    "result_filenames": ["/path/to/csv/with/results"],
    "results_path": "/path/to/results",
    "eval_path": "/path/to/eval/folder",
    "datasets_path": None,  # config.py: $BOP_PATH, read when the arguments are parsed
    "targets_filename": "test_targets_bop19.json",
    "out_errors_tpath": os.path.join("{eval_path}", "{result_name}", "{error_sign}",
                                     "errors_{scene_id:06d}.json"),
}

POINT_ERRORS = ("ad", "add", "adi", "mssd", "mspd", "proj")
# VSD batches whose distinct renders number at most this times the tuples take
# the shared-render path (batch.BatchEvaluator.vsd_shared); one instance per
# object (2 renders per tuple) keeps the fused per-tuple kernel
SHARED_RENDER_RATIO = float(os.environ.get("BOPX_SHARED_RENDER_RATIO", "1.5"))


def depth_group_frames():
  """VSD test depth of consecutive scenes is decoded in shared k_png_inflate
  launches of about this many frames (depth_gpu.GroupPrefetch;
  BOPX_DEPTH_GROUP_FRAMES=0: one launch per scene, from the scene prefetch;
  "G/F": groups of G frames, the first one of F; default 4096/1024: the error
  kernels start on a small first group while the next ones decode)."""
  return depth_group_sizes()[0]


def depth_group_sizes():
  """(group frames, first group frames) from BOPX_DEPTH_GROUP_FRAMES."""
  v = os.environ.get("BOPX_DEPTH_GROUP_FRAMES", "4096/1024").split("/")
  g = int(v[0])
  return g, (int(v[1]) if len(v) > 1 else g)


def release_group_slice(groups, scene_id):
  """Take a scene's slice of its decode group without using it (a scene with
  no VSD tuples), so the group can be freed once its last scene is taken. The
  frames are never read, so whatever the group failed with (a frame of another
  size in another scene of the group, ...) is not this scene's error: the
  reference reads every target image's depth (eval_calc_errors.py:238-243) but
  uses it only per estimate, where a size mismatch would surface. The scenes
  of the group that do use their frames still get the group's error (and fall
  back to per-scene decoding on ValueError). ADVICE r5."""
  try:
    groups.get(scene_id)
  except Exception:  # noqa: BLE001 - frames unused; the scenes that need them re-raise
    pass


ERROR_TYPES = ("vsd", "mssd", "mspd", "ad", "add", "adi", "cus", "proj", "rete", "re", "te")


def parse_args(argv=None):
  """The reference's command line (eval_calc_errors.py:89-129), same
  defaults and the same string-to-type conversions."""
  p = copy.deepcopy(DEFAULTS)
  p["datasets_path"] = os.environ.get("BOP_PATH", "/path/to/bop/datasets")
  ap = argparse.ArgumentParser()
  ap.add_argument("--n_top", default=p["n_top"])
  ap.add_argument("--error_type", default=p["error_type"])
  ap.add_argument("--vsd_deltas",
                  default=",".join("{}:{}".format(k, v) for k, v in p["vsd_deltas"].items()))
  ap.add_argument("--vsd_taus", default=",".join(map(str, p["vsd_taus"])))
  ap.add_argument("--vsd_normalized_by_diameter", default=p["vsd_normalized_by_diameter"])
  ap.add_argument("--max_sym_disc_step", default=p["max_sym_disc_step"])
  ap.add_argument("--skip_missing", default=p["skip_missing"])
  ap.add_argument("--renderer_type", default=p["renderer_type"])
  ap.add_argument("--result_filenames", default=",".join(p["result_filenames"]))
  ap.add_argument("--results_path", default=p["results_path"])
  ap.add_argument("--eval_path", default=p["eval_path"])
  ap.add_argument("--datasets_path", default=p["datasets_path"])
  ap.add_argument("--targets_filename", default=p["targets_filename"])
  ap.add_argument("--out_errors_tpath", default=p["out_errors_tpath"])
  a = ap.parse_args(argv)
  p["n_top"] = int(a.n_top)
  p["error_type"] = str(a.error_type)
  p["vsd_deltas"] = {str(e.split(":")[0]): float(e.split(":")[1])
                     for e in a.vsd_deltas.split(",")}
  p["vsd_taus"] = list(map(float, a.vsd_taus.split(",")))
  p["vsd_normalized_by_diameter"] = bool(a.vsd_normalized_by_diameter)
  p["max_sym_disc_step"] = float(a.max_sym_disc_step)
  p["skip_missing"] = bool(a.skip_missing)
  p["renderer_type"] = str(a.renderer_type)
  p["result_filenames"] = a.result_filenames.split(",")
  for k in ("results_path", "eval_path", "datasets_path", "targets_filename",
            "out_errors_tpath"):
    p[k] = str(getattr(a, k))
  return p


def log(s):
  misc.log(s)


# Parsed annotation / model / result files, shared by the error types of one
# process (eval_bop19_pose runs VSD, MSSD and MSPD over the same files): keyed
# by path, size and mtime, so an edited file is read again. Callers treat the
# returned objects as read-only.
_FILE_CACHE = {}
_FILE_CACHE_MAX = 512
_KEY_LOCKS = {}
_KEY_LOCKS_LOCK = threading.Lock()


def _key_lock(key):
  """One lock per cache key: a file (or a scene's arrays) requested by two
  threads at once (the scene prefetch and the depth-group thread) is parsed
  once and both get the same object (the identity-keyed caches rely on it)."""
  with _KEY_LOCKS_LOCK:
    lk = _KEY_LOCKS.get(key)
    if lk is None:
      if len(_KEY_LOCKS) >= 8192:
        _KEY_LOCKS.clear()
      lk = _KEY_LOCKS[key] = threading.Lock()
    return lk


def cached_load(loader, path, **kw):
  st = os.stat(path)
  key = (loader.__name__, os.path.abspath(path), st.st_size, st.st_mtime_ns,
         tuple(sorted(kw.items())))
  hit = _FILE_CACHE.get(key)
  if hit is None:
    with _key_lock(key):
      hit = _FILE_CACHE.get(key)
      if hit is None:
        if len(_FILE_CACHE) >= _FILE_CACHE_MAX:
          _FILE_CACHE.pop(next(iter(_FILE_CACHE)))
        with inout.gc_paused():  # parsed files are acyclic
          hit = _FILE_CACHE[key] = loader(path, **kw)
  return hit


def scene_gt_arrays(path):
  """A scene's GT for the arrays path: load_scene_gt_lists' GTLists (cached
  like any parse), or load_scene_gt's dict when the native reader declines
  the file."""
  g = cached_load(inout.load_scene_gt_lists, path)
  return g if g is not None else cached_load(inout.load_scene_gt, path)


# ----------------------------------------------------------------- enumeration
_ORG_CACHE = {}


def organize(targets, ests):
  """targets_org[scene][im][obj] = target; ests_org[scene][im][obj] = [est]
  (insertion order, eval_calc_errors.py:207-228). The parsed files come from
  cached_load (the same objects for every error type of a BOP19 run), so the
  organised view is cached on their identity too; callers treat it as read-only."""
  key = (id(targets), id(ests))
  hit = _ORG_CACHE.get(key)
  if hit is not None and hit[0] is targets and hit[1] is ests:
    return hit[2]
  with inout.gc_paused():
    out = _organize(targets, ests)
  if len(_ORG_CACHE) > 8:
    _ORG_CACHE.clear()
  _ORG_CACHE[key] = (targets, ests, out)
  return out


def _organize(targets, ests):
  targets_org, ests_org = {}, {}
  for t in targets:
    targets_org.setdefault(t["scene_id"], {}).setdefault(t["im_id"], {})[t["obj_id"]] = t
  for e in ests:
    ests_org.setdefault(e["scene_id"], {}).setdefault(e["im_id"], {}).setdefault(
        e["obj_id"], []).append(e)
  return targets_org, ests_org


def scene_records(p, scene_id, scene_targets, ests_org, scene_gt):
  """The records of one scene in output order, each with the GT ids it is
  evaluated against (eval_calc_errors.py:238-290)."""
  recs = []
  n_ests = 0
  for im_id, im_targets in scene_targets.items():
    for obj_id, target in im_targets.items():
      if p["n_top"] == 0:
        n_top = None
      elif p["n_top"] == -1:
        n_top = target["inst_count"]
      else:
        n_top = p["n_top"]
      obj_ests = ests_org.get(scene_id, {}).get(im_id, {}).get(obj_id, [])
      if not p["skip_missing"] and len(obj_ests) < n_top:
        raise ValueError(
            "Not enough estimates for scene: {}, im: {}, obj: {} (provided: {}, expected: {})"
            .format(scene_id, im_id, obj_id, len(obj_ests), n_top))
      ranked = sorted(enumerate(obj_ests), key=lambda x: x[1]["score"], reverse=True)
      ranked = ranked[slice(0, n_top)]
      n_ests += len(ranked)
      gts = [(gt_id, gt) for gt_id, gt in enumerate(scene_gt[im_id]) if gt["obj_id"] == obj_id]
      for est_id, est in ranked:
        recs.append({"im_id": im_id, "obj_id": obj_id, "est_id": est_id, "score": est["score"],
                     "R": est["R"], "t": est["t"], "gts": gts})
  return recs, n_ests


_REC_CACHE = {}


def scene_records_cached(p, scene_id, scene_targets, ests_org, scene_gt):
  """scene_records, shared by the error types of one BOP19 run: the inputs are
  the cached parses (the same objects for every error type), so the records
  are keyed on their identity and the n_top / skip_missing settings; callers
  treat them as read-only."""
  key = (scene_id, id(scene_targets), id(ests_org), id(scene_gt), p["n_top"], p["skip_missing"])
  hit = _REC_CACHE.get(key)
  if hit is not None and hit[0] is scene_targets and hit[1] is ests_org and hit[2] is scene_gt:
    return hit[3]
  out = scene_records(p, scene_id, scene_targets, ests_org, scene_gt)
  if len(_REC_CACHE) >= 4096:
    _REC_CACHE.clear()
  _REC_CACHE[key] = (scene_targets, ests_org, scene_gt, out)
  return out


def gate(error_type, diameter, t_e, t_g):
  """Host pre-check of one tuple: None = evaluate, else the fill value list
  (eval_calc_errors.py:292-339). n_tau is applied by the caller for VSD."""
  if error_type in ("vsd", "cus"):
    if not misc.overlapping_sphere_projections(0.5 * diameter, t_e.squeeze(), t_g.squeeze()):
      return "vsd_fill"
  elif error_type in ("ad", "add", "adi", "mssd"):
    if not np.linalg.norm(t_e - t_g) < diameter:
      return [float("inf")]
  return None


# ------------------------------------------------------------------ evaluation
_SYM_CACHE = {}  # (step, discrete, continuous) -> S x 12 symmetry rows


def symmetry_rows(info, step):
  """misc.get_symmetry_transformations(info, step) as S x 12 rows
  (misc.symmetries_to_array), cached for the process on the model info's
  symmetry fields and the step."""
  key = (float(step), repr(info.get("symmetries_discrete")),
         repr(info.get("symmetries_continuous")))
  hit = _SYM_CACHE.get(key)
  if hit is None:
    with _key_lock(("sym",) + key):
      hit = _SYM_CACHE.get(key)
      if hit is None:
        if len(_SYM_CACHE) >= 4096:
          _SYM_CACHE.clear()
        hit = _SYM_CACHE[key] = misc.symmetries_to_array(
            misc.get_symmetry_transformations(info, step))
  return hit


def prefetch_symmetries(models_info_path, step):
  """Start computing every object's symmetry rows on a thread (the BOP19 run
  needs them for MSSD / MSPD after its VSD pass); returns the thread."""
  def work():
    try:
      info = cached_load(inout.load_json, models_info_path, keys_to_int=True)
      for v in info.values():
        if isinstance(v, dict):
          symmetry_rows(v, step)
    except Exception:  # noqa: BLE001 - the passes compute what is missing themselves
      pass
  t = threading.Thread(target=work, name="bopx-symmetries", daemon=True)
  t.start()
  return t


class Models:
  """Objects of one dataset resident on the GPU (+ host-side info).

  The evaluator (evaluator(device)) keeps its objects between runs: an object
  whose model file (path, size, mtime) and diameter are unchanged is not
  uploaded again, and its symmetry set is only (re)computed when the error
  type needs one that is not registered yet (VSD -> MSSD -> MSPD of one BOP19
  run: one upload per model, one symmetry set per object). Objects of other
  models are removed, so ev.objects is exactly this dataset's."""

  def __init__(self, ev, p, dp_model, models_info):
    self.ev = ev
    self.info = models_info
    need_syms = p["error_type"] in ("mssd", "mspd")
    self.sym_ids = set(dp_model["symmetric_obj_ids"] or [])
    reg = ev.__dict__.setdefault("_bopx_reg", {})  # obj_id -> (mesh key, symmetry key)
    keep = set()
    pending = []  # (obj_id, symmetry rows, keys) of resident objects: one upload call
    for obj_id in dp_model["obj_ids"]:
      path = dp_model["model_tpath"].format(obj_id=obj_id)
      if not os.path.exists(path):
        continue
      st = os.stat(path)
      dia = models_info[obj_id]["diameter"] if models_info is not None else None
      mkey = (os.path.abspath(path), st.st_size, st.st_mtime_ns, dia)
      skey = None
      if need_syms:
        info = models_info[obj_id]
        skey = (p["max_sym_disc_step"], repr(info.get("symmetries_discrete")),
                repr(info.get("symmetries_continuous")))
      have = reg.get(obj_id)
      keep.add(obj_id)
      if have is not None and have[0] == mkey and obj_id in ev.objects:
        if need_syms and have[1] != skey:
          pending.append((obj_id, symmetry_rows(models_info[obj_id], p["max_sym_disc_step"]),
                          (mkey, skey)))
        continue
      if obj_id in ev.objects:
        ev.remove_object(obj_id)
      m = cached_load(inout.load_ply, path)
      syms = None
      if need_syms:
        syms = symmetry_rows(models_info[obj_id], p["max_sym_disc_step"])
      ev.add_object(obj_id, m["pts"], m.get("faces"), syms, dia)
      reg[obj_id] = (mkey, skey)
    if pending:
      many = getattr(ev, "set_symmetries_many", None)
      if many is not None:
        many([(o, s) for o, s, _ in pending])
      else:
        for o, s, _ in pending:
          ev.set_symmetries(o, s)
      for o, _, keys in pending:
        reg[o] = keys
    for obj_id in [o for o in ev.objects if o not in keep]:
      ev.remove_object(obj_id)
      reg.pop(obj_id, None)


_EVALUATORS = {}  # device -> BatchEvaluator, shared by the runs of one process


def evaluator(device):
  from .batch import BatchEvaluator
  ev = _EVALUATORS.get(int(device))
  if ev is None:
    ev = _EVALUATORS[int(device)] = BatchEvaluator(device)
  return ev


def _pose12(R, t):
  return np.concatenate([np.asarray(R, np.float64).reshape(9),
                         np.asarray(t, np.float64).reshape(3)])


def _poses12(Rs, ts):
  """[n, 12] float64 rows [R row-major | t] of n poses (_pose12 per pose, in one
  conversion when the shapes agree)."""
  n = len(Rs)
  try:
    return np.concatenate([np.asarray(Rs, np.float64).reshape(n, 9),
                           np.asarray(ts, np.float64).reshape(n, 3)], 1)
  except ValueError:
    return np.stack([_pose12(R, t) for R, t in zip(Rs, ts)]).reshape(n, 12)


def gates(error_type, dias, t_es, t_gs):
  """gate() of many tuples at once: bool array, True = filled (not evaluated).
  The sphere-projection / distance tests run vectorised; a tuple within a
  relative 1e-9 of its threshold (or with a zero depth, NaN, ...) is decided by
  the scalar gate(), so the result is gate()'s for every tuple."""
  n = len(t_es)
  fill = np.zeros(n, bool)
  if n == 0 or error_type not in ("vsd", "cus", "ad", "add", "adi", "mssd"):
    return fill
  te = np.asarray(t_es, np.float64).reshape(n, 3)
  tg = np.asarray(t_gs, np.float64).reshape(n, 3)
  dia = np.asarray(dias, np.float64)
  with np.errstate(all="ignore"):
    if error_type in ("vsd", "cus"):
      d = te[:, :2] / te[:, 2:3] - tg[:, :2] / tg[:, 2:3]
      val = np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1])
      thr = (0.5 * dia) * (1.0 / te[:, 2] + 1.0 / tg[:, 2])
    else:
      e = te - tg
      val = np.sqrt((e * e).sum(1))
      thr = dia
    fill = ~(val < thr)
    sure = np.abs(val - thr) > 1e-9 * np.maximum(np.abs(val), np.abs(thr))
    if error_type in ("vsd", "cus"):
      sure &= (te[:, 2] != 0) & (tg[:, 2] != 0)
  for i in np.nonzero(~sure)[0]:
    fill[i] = gate(error_type, float(dia[i]), np.asarray(t_es[i]), np.asarray(t_gs[i])) is not None
  return fill


def plan(p, recs, models_info):
  """Host gates of every (record, GT) pair: errs with the filled values and
  None placeholders, and the todo list [(record, gt_id, R_g, t_g)] for the GPU."""
  et = p["error_type"]
  n_tau = len(p["vsd_taus"])
  errs = [dict() for _ in recs]
  todo = []
  pairs = [(ri, gt_id, gt) for ri, r in enumerate(recs) for gt_id, gt in r["gts"]]
  fills = None
  if models_info is not None and et in ("vsd", "cus", "ad", "add", "adi", "mssd"):
    fills = gates(et, [models_info[recs[ri]["obj_id"]]["diameter"] for ri, _, _ in pairs],
                  [recs[ri]["t"] for ri, _, _ in pairs], [gt["cam_t_m2c"] for _, _, gt in pairs])
  for k, (ri, gt_id, gt) in enumerate(pairs):
    r = recs[ri]
    R_g, t_g = gt["cam_R_m2c"], gt["cam_t_m2c"]
    if fills is not None:
      fill = None
      if fills[k]:
        fill = "vsd_fill" if et in ("vsd", "cus") else [float("inf")]
    else:
      dia = models_info[r["obj_id"]]["diameter"] if models_info is not None else None
      fill = gate(et, dia, r["t"], t_g)
    if fill == "vsd_fill":
      errs[ri][gt_id] = [1.0] * (n_tau if et == "vsd" else 1)
    elif fill is not None:
      errs[ri][gt_id] = fill
    elif et in ("re", "te", "rete"):
      e_re = pose_error.re(r["R"], R_g)
      e_te = pose_error.te(r["t"], t_g)
      errs[ri][gt_id] = {"re": [e_re], "te": [e_te], "rete": [e_re, e_te]}[et]
    else:
      errs[ri][gt_id] = None  # filled from the GPU batch
      todo.append((ri, gt_id, R_g, t_g))
  return errs, todo


def row_to_errors(et, row):
  """Error list of one tuple from its raw batch row (VSD: n_tau values, CUS:
  the silhouette-overlap row, others: one value)."""
  if et == "vsd":
    return [float(v) for v in row]
  if et == "cus":
    return [pose_error.cus_from_cover(row)]
  return [float(row[0])]


def todo_images(recs, todo):
  """Sorted image ids of the tuples in todo (one test-depth frame each)."""
  return sorted({recs[ri]["im_id"] for ri, _, _, _ in todo})


_PINNED = [None]  # the page-locked staging buffer reused by load_scene_depths(reuse=True)


def scene_depth_paths(dp_split, scene_camera, scene_id, ims):
  """Depth PNG paths and depth_scale values of the images ims (:240-243)."""
  paths = [dp_split["depth_tpath"].format(scene_id=scene_id, im_id=im_id) for im_id in ims]
  return paths, [scene_camera[im_id]["depth_scale"] for im_id in ims]


def load_scene_depths(dp_split, scene_camera, scene_id, ims, torch=None, reuse=False):
  """Test depth of the images ims in mm, float32 (eval_calc_errors.py:240-243),
  decoded straight into one (n, H, W) array — page-locked when torch is given,
  so the upload to the GPU is one DMA — or a list when the sizes differ.
  reuse: the frames land in one page-locked buffer kept across calls (grown
  when needed; page-locking a scene's 1-2 GB anew per scene is slow), valid
  until the next such call — the caller uploads and synchronises first."""
  paths, scales = scene_depth_paths(dp_split, scene_camera, scene_id, ims)  # float32, :242-243
  W, H = dp_split["im_size"]
  if torch is not None and torch.cuda.is_available() and os.environ.get("BOPX_PIN", "1") != "0":
    if reuse:
      need = len(ims) * H * W
      if _PINNED[0] is None or _PINNED[0].numel() < need:
        _PINNED[0] = None
        _PINNED[0] = torch.empty(max(need, 1), dtype=torch.float32, pin_memory=True)
      buf = _PINNED[0][:need].view(len(ims), H, W)
    else:
      buf = torch.empty((len(ims), H, W), dtype=torch.float32, pin_memory=True)
    try:
      inout.load_depths(paths, scales=scales, out=buf.numpy())
      return buf
    except ValueError:
      pass  # a frame of another size: per-frame arrays below
  buf = np.empty((len(ims), H, W), np.float32)
  try:
    return inout.load_depths(paths, scales=scales, out=buf)
  except ValueError:
    return inout.load_depths(paths, scales=scales)


def _vsd_launch(ev, torch, p, dataset, slots, d_pe, d_pg, obj, pe, pg, fidx_h, fidx, cam, depths,
                models_info):
  """The GPU VSD rows of one scene batch: the fused kernel, or shared renders
  for multi-instance batches (SHARED_RENDER_RATIO)."""
  n = len(obj)
  dev = ev.device
  T = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
  if isinstance(depths, list):
    depths = np.stack(depths)
  d_frames = depths.to(dev, non_blocking=True) if torch.is_tensor(depths) else T(depths, torch.float32)
  dia = np.array([models_info[o]["diameter"] for o in obj], np.float64)
  delta = p["vsd_deltas"][dataset]
  from . import runtime
  from .batch import unique_renders
  # multi-instance images (every estimate x every GT instance of its object,
  # :281-290): each distinct pose rendered once when that saves renders
  # one tuple per (image, object) (single-instance data): 2 n renders, fused path
  single = len(np.unique(fidx_h.astype(np.int64) << 32 | obj.astype(np.int64))) == n
  ro, rp, rf, er, gr = (None,) * 5 if single and SHARED_RENDER_RATIO < 2 else \
      unique_renders(obj, pe, pg, fidx_h)
  if ro is not None and len(ro) <= SHARED_RENDER_RATIO * n:
    from ._lib import BopxOOMError
    try:
      return ev.vsd_shared(ev.slots(ro), T(rp, torch.float64), T(rf, torch.int32),
                           T(er, torch.int32), T(gr, torch.int32), d_frames,
                           T(cam, torch.float64), delta, p["vsd_taus"], T(dia, torch.float64),
                           normalized_by_diameter=p["vsd_normalized_by_diameter"],
                           cost_type="step", delta_flags=runtime.delta_flags(delta))
    except BopxOOMError:
      # the shared path's ROI-sized depth buffers (outside torch's caching
      # allocator) did not fit: the fused kernel needs no such scratch and
      # gives the same rows bit for bit
      torch.cuda.empty_cache()
  return ev.vsd(slots, d_pe, d_pg, fidx, d_frames,
                T(cam, torch.float64), delta, p["vsd_taus"], T(dia, torch.float64),
                normalized_by_diameter=p["vsd_normalized_by_diameter"], cost_type="step",
                delta_flags=runtime.delta_flags(delta))


def evaluate_batch(ev, torch, p, dataset, dp_split, scene_camera, scene_id, recs, models_info,
                   symmetric_ids, todo, depths=None):
  """Raw float64 rows [len(todo), C] of the GPU evaluation of todo (depths:
  the frames of todo_images(recs, todo), or None to load them here)."""
  et = p["error_type"]
  dev = ev.device
  n = len(todo)
  obj = np.array([recs[ri]["obj_id"] for ri, _, _, _ in todo], np.int32)
  pe = _poses12([recs[ri]["R"] for ri, _, _, _ in todo], [recs[ri]["t"] for ri, _, _, _ in todo])
  pg = _poses12([R_g for _, _, R_g, _ in todo], [t_g for _, _, _, t_g in todo])
  T = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
  slots = ev.slots(obj)
  d_pe, d_pg = T(pe, torch.float64), T(pg, torch.float64)
  if et in ("vsd", "cus"):
    ims = todo_images(recs, todo)
    frame_of = {im: k for k, im in enumerate(ims)}
    cam = np.array([[K[0, 0], K[1, 1], K[0, 2], K[1, 2]]
                    for K in (scene_camera[im]["cam_K"] for im in ims)], np.float64)
    fidx_h = np.array([frame_of[recs[ri]["im_id"]] for ri, _, _, _ in todo], np.int32)
    fidx = T(fidx_h, torch.int32)
    if et == "cus":
      W, H = dp_split["im_size"]
      return ev.cover(slots, d_pe, d_pg, fidx, T(cam, torch.float64), W, H)
    if depths is None:
      depths = load_scene_depths(dp_split, scene_camera, scene_id, ims, torch)
    return _vsd_launch(ev, torch, p, dataset, slots, d_pe, d_pg, obj, pe, pg, fidx_h, fidx, cam,
                       depths, models_info)
  if et in ("mspd", "proj"):
    K = np.stack([scene_camera[recs[ri]["im_id"]]["cam_K"].reshape(9) for ri, _, _, _ in todo])
    fn = ev.mspd if et == "mspd" else ev.proj
    return fn(slots, d_pe, d_pg, T(K, torch.float64)).view(n, 1)
  if et == "mssd":
    return ev.mssd(slots, d_pe, d_pg).view(n, 1)
  if et in ("ad", "add", "adi"):
    use_adi = np.array([et == "adi" or (et == "ad" and int(o) in symmetric_ids) for o in obj])
    out = torch.empty(n, dtype=torch.float64, device=dev)
    for flag, fn in ((False, ev.add), (True, ev.adi)):
      idx = np.nonzero(use_adi == flag)[0]
      if len(idx):
        ii = T(idx, torch.int64)
        out[ii] = fn(slots[ii], d_pe[ii], d_pg[ii])
    return out.view(n, 1)
  raise ValueError("Unknown pose error function.")


# ---------------------------------------------------- array path (BOP19 types)
# The error types of a BOP19 evaluation (VSD, MSSD, MSPD) on one process: the
# records of a scene and their (record, GT) pairs as arrays, the gates and the
# GPU rows written into one values array, the errors files by the native
# writer (inout.save_errors_arrays): no per-tuple Python dicts. The same tuples,
# fills and bytes as plan / evaluate / save_json (tests/test_e2e_errors.py);
# BOPX_ERRORS_ARRAYS=0 takes the record-dict path.
ARRAY_TYPES = ("vsd", "mssd", "mspd")


def scene_arrays(recs):
  """Records of a scene (scene_records) as arrays: rec_im / rec_obj / rec_est
  int64, rec_score float64, pose [n_rec, 12]; their GT pairs in record order
  (ascending GT id) pair_off [n_rec + 1], pair_ri, pair_gt, pg [n_pairs, 12]."""
  n = len(recs)
  rec_im = np.fromiter((r["im_id"] for r in recs), np.int64, n)
  rec_obj = np.fromiter((r["obj_id"] for r in recs), np.int64, n)
  rec_est = np.fromiter((r["est_id"] for r in recs), np.int64, n)
  rec_score = np.fromiter((r["score"] for r in recs), np.float64, n)
  cnt = np.fromiter((len(r["gts"]) for r in recs), np.int64, n)
  pair_off = np.zeros(n + 1, np.int64)
  np.cumsum(cnt, out=pair_off[1:])
  m = int(pair_off[-1])
  pair_ri = np.repeat(np.arange(n, dtype=np.int64), cnt)
  pair_gt = np.fromiter((g for r in recs for g, _ in r["gts"]), np.int64, m)
  pe = _poses12([r["R"] for r in recs], [r["t"] for r in recs]) if n else np.zeros((0, 12))
  pg = _poses12([gt["cam_R_m2c"] for r in recs for _, gt in r["gts"]],
                [gt["cam_t_m2c"] for r in recs for _, gt in r["gts"]]) if m else np.zeros((0, 12))
  return {"rec_im": rec_im, "rec_obj": rec_obj, "rec_est": rec_est, "rec_score": rec_score,
          "pe": pe, "pair_off": pair_off, "pair_ri": pair_ri, "pair_gt": pair_gt, "pg": pg}


def scene_arrays_direct(p, scene_id, scene_targets, ests_org, scene_gt):
  """scene_arrays(scene_records(...)) without the per-record dicts (the arrays
  path keeps no records): the same traversal, ranking, n_top rule, errors and
  GT pairs (eval_calc_errors.py:238-290), straight into lists. Returns
  (arrays, n_ests). scene_gt: load_scene_gt's dict or load_scene_gt_lists'
  GTLists (the same pairs and rows)."""
  n_top_p, skip = p["n_top"], p["skip_missing"]
  se = ests_org.get(scene_id, {})
  rec_im, rec_obj, rec_est, rec_score, est_R, est_t, cnt = [], [], [], [], [], [], []
  pair_gt, gt_R, gt_t, pair_row = [], [], [], []
  lists = isinstance(scene_gt, inout.GTLists)  # the native reader's arrays (load_scene_gt_lists)
  gl_obj = scene_gt.obj.tolist() if lists else None
  for im_id, im_targets in scene_targets.items():
    ie = se.get(im_id, {})
    for obj_id, target in im_targets.items():
      if n_top_p == 0:
        n_top = None
      elif n_top_p == -1:
        n_top = target["inst_count"]
      else:
        n_top = n_top_p
      obj_ests = ie.get(obj_id, [])
      if not skip and len(obj_ests) < n_top:
        raise ValueError(
            "Not enough estimates for scene: {}, im: {}, obj: {} (provided: {}, expected: {})"
            .format(scene_id, im_id, obj_id, len(obj_ests), n_top))
      ranked = sorted(enumerate(obj_ests), key=lambda x: x[1]["score"], reverse=True)
      ranked = ranked[slice(0, n_top)]
      if lists:
        a, b = scene_gt.rows(im_id)
        gts = [g for g, o in enumerate(gl_obj[a:b]) if o == obj_id]
      else:
        gts = [(gt_id, gt) for gt_id, gt in enumerate(scene_gt[im_id]) if gt["obj_id"] == obj_id]
      for est_id, est in ranked:
        rec_im.append(im_id)
        rec_obj.append(obj_id)
        rec_est.append(est_id)
        rec_score.append(est["score"])
        est_R.append(est["R"])
        est_t.append(est["t"])
        cnt.append(len(gts))
        if lists:
          pair_gt.extend(gts)
          pair_row.extend(a + g for g in gts)
          continue
        for gt_id, gt in gts:
          pair_gt.append(gt_id)
          gt_R.append(gt["cam_R_m2c"])
          gt_t.append(gt["cam_t_m2c"])
  n, m = len(rec_im), len(pair_gt)
  if lists and m:  # the rows load_scene_gt's arrays give (_poses12: R row-major | t)
    rows = np.asarray(pair_row, np.int64)
    pg = np.concatenate([scene_gt.fields["cam_R_m2c"][rows], scene_gt.fields["cam_t_m2c"][rows]], 1)
  else:
    pg = _poses12(gt_R, gt_t) if m else np.zeros((0, 12))
  cnt = np.array(cnt, np.int64).reshape(n)
  pair_off = np.zeros(n + 1, np.int64)
  np.cumsum(cnt, out=pair_off[1:])
  arr = {"rec_im": np.array(rec_im, np.int64).reshape(n),
         "rec_obj": np.array(rec_obj, np.int64).reshape(n),
         "rec_est": np.array(rec_est, np.int64).reshape(n),
         "rec_score": np.array(rec_score, np.float64).reshape(n),
         "pe": _poses12(est_R, est_t) if n else np.zeros((0, 12)), "pair_off": pair_off,
         "pair_ri": np.repeat(np.arange(n, dtype=np.int64), cnt),
         "pair_gt": np.array(pair_gt, np.int64).reshape(m),
         "pg": pg}
  return arr, n


_DIRECT_CACHE = {}


def scene_arrays_direct_cached(p, scene_id, scene_targets, ests_org, scene_gt):
  """scene_arrays_direct shared by the error types of one BOP19 run (keyed like
  scene_records_cached; callers treat the arrays as read-only)."""
  key = (scene_id, id(scene_targets), id(ests_org), id(scene_gt), p["n_top"], p["skip_missing"])
  with _key_lock(("direct",) + key):
    hit = _DIRECT_CACHE.get(key)
    if hit is not None and hit[0] is scene_targets and hit[1] is ests_org and hit[2] is scene_gt:
      return hit[3]
    out = scene_arrays_direct(p, scene_id, scene_targets, ests_org, scene_gt)
    if len(_DIRECT_CACHE) >= 4096:
      _DIRECT_CACHE.clear()
    _DIRECT_CACHE[key] = (scene_targets, ests_org, scene_gt, out)
    return out


_ARR_CACHE = {}


def scene_arrays_cached(recs):
  """scene_arrays, shared by the error types of one BOP19 run (recs is the
  cached record list: keyed on its identity)."""
  hit = _ARR_CACHE.get(id(recs))
  if hit is not None and hit[0] is recs:
    return hit[1]
  out = scene_arrays(recs)
  if len(_ARR_CACHE) >= 4096:
    _ARR_CACHE.clear()
  _ARR_CACHE[id(recs)] = (recs, out)
  return out


def plan_arrays(p, arr, models_info):
  """plan() on the arrays: the values array [n_pairs, n_values] with the gate
  fills (VSD 1.0, MSSD inf; MSPD ungated, :296-339) and the pair indices left
  for the GPU."""
  et = p["error_type"]
  nv = len(p["vsd_taus"]) if et == "vsd" else 1
  m = len(arr["pair_gt"])
  vals = np.empty((m, nv), np.float64)
  fill = np.zeros(m, bool)
  if m and et in ("vsd", "mssd"):
    objs, inv = np.unique(arr["rec_obj"][arr["pair_ri"]], return_inverse=True)
    dia = np.array([models_info[o]["diameter"] for o in objs.tolist()], np.float64)[inv]
    fill = gates(et, dia, arr["pe"][arr["pair_ri"], 9:12], arr["pg"][:, 9:12])
    vals[fill] = 1.0 if et == "vsd" else float("inf")
  return vals, np.nonzero(~fill)[0]


def evaluate_batch_arrays(ev, torch, p, dataset, dp_split, scene_camera, scene_id, arr, todo,
                          models_info, depths=None, depth_ims=None):
  """evaluate_batch on the arrays: the GPU rows [len(todo), n_values] of the
  pairs todo (depths: the frames of their sorted images, or None; with
  depth_ims, the frames of those sorted image ids, a superset)."""
  et = p["error_type"]
  dev = ev.device
  ri = arr["pair_ri"][todo]
  obj = arr["rec_obj"][ri].astype(np.int32)
  pe, pg = arr["pe"][ri], arr["pg"][todo]
  T = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
  slots = ev.slots(obj)
  d_pe, d_pg = T(pe, torch.float64), T(pg, torch.float64)
  ims, inv = np.unique(arr["rec_im"][ri], return_inverse=True)  # todo_images order
  Ks = [np.asarray(scene_camera[im]["cam_K"], np.float64).reshape(3, 3) for im in ims.tolist()]
  if et == "vsd":
    if depths is not None and depth_ims is not None:
      depth_ims = np.asarray(depth_ims, np.int64)
      pos = np.searchsorted(depth_ims, ims)
      if len(ims) and (pos.max() >= len(depth_ims) or not np.array_equal(depth_ims[pos], ims)):
        raise ValueError("depth frames do not cover the batch's images")
      Ks = [np.asarray(scene_camera[im]["cam_K"], np.float64).reshape(3, 3)
            for im in depth_ims.tolist()]
      inv = pos[inv]
    cam = np.array([[K[0, 0], K[1, 1], K[0, 2], K[1, 2]] for K in Ks], np.float64)
    fidx_h = inv.astype(np.int32)
    if depths is None:
      depths = load_scene_depths(dp_split, scene_camera, scene_id, ims.tolist(), torch)
    return _vsd_launch(ev, torch, p, dataset, slots, d_pe, d_pg, obj, pe, pg, fidx_h,
                       T(fidx_h, torch.int32), cam, depths, models_info)
  if et == "mspd":
    K = np.stack([K.reshape(9) for K in Ks])[inv]
    return ev.mspd(slots, d_pe, d_pg, T(K, torch.float64)).view(len(todo), 1)
  return ev.mssd(slots, d_pe, d_pg).view(len(todo), 1)


def _dist():
  import torch.distributed as dist
  if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
    return dist.get_rank(), dist.get_world_size()
  return 0, 1


def todo_costs(objects, p, recs, todo, scene_camera, im_size):
  """Estimated cost of every todo tuple for the LPT image shard (SURVEY.md §8d
  flop model, shard.error_cost): mesh size, symmetry count and, for VSD / CUS,
  the tuple's ROI (bbox corners of the model in both poses, projected with the
  image's K). objects: BatchEvaluator.objects (nv, nf, ns, bbox per obj_id).
  None when the object table is not available (uniform weights)."""
  from . import shard
  if not todo or not objects:
    return None
  et = p["error_type"]
  obj = [recs[ri]["obj_id"] for ri, _, _, _ in todo]
  o = [objects[i] for i in obj]
  nv = np.array([x["nv"] for x in o], np.float64)
  nf = np.array([x["nf"] for x in o], np.float64)
  ns = np.array([max(1, x["ns"]) for x in o], np.float64)
  roi = np.zeros(len(todo))
  if et in ("vsd", "cus") and scene_camera is not None:
    lo = np.stack([x["bbox"][0] for x in o])
    hi = np.stack([x["bbox"][1] for x in o])
    pe = _poses12([recs[ri]["R"] for ri, _, _, _ in todo],
                  [recs[ri]["t"] for ri, _, _, _ in todo])
    pg = _poses12([R_g for _, _, R_g, _ in todo], [t_g for _, _, _, t_g in todo])
    K = np.stack([np.asarray(scene_camera[recs[ri]["im_id"]]["cam_K"], np.float64).reshape(3, 3)
                  for ri, _, _, _ in todo])
    roi = shard.roi_pixels(lo, hi, [pe, pg], K, im_size[0], im_size[1])
  return shard.error_cost(et, nv, nf, ns, roi)


def shard_todo(recs, todo, world, costs=None):
  """Images of the scene over ranks (LPT on the summed `costs` of each image's
  todo entries, or on its tuple count); returns one index array into todo per
  rank (possibly empty: fewer images than ranks)."""
  from . import shard
  ims = sorted({recs[ri]["im_id"] for ri, _, _, _ in todo})
  col = {im: k for k, im in enumerate(ims)}
  frame = np.array([col[recs[ri]["im_id"]] for ri, _, _, _ in todo])
  w = np.ones(len(todo)) if costs is None else np.asarray(costs, np.float64)
  parts = shard.lpt_shard(shard.image_costs(frame, w, len(ims)), world)
  return [np.nonzero(np.isin(frame, part))[0] for part in parts]


def plan_rank(p, recs, models_info, objects, scene_camera, im_size, rank, world):
  """plan() plus this rank's LPT share of the todo tuples (all of them for one
  rank): (errs, todo, mine)."""
  errs, todo = plan(p, recs, models_info)
  if world == 1 or not todo:
    return errs, todo, np.arange(len(todo))
  costs = todo_costs(objects, p, recs, todo, scene_camera, im_size)
  return errs, todo, shard_todo(recs, todo, world, costs)[rank]


def evaluate(ev, torch, p, dataset, dp_split, scene_camera, scene_id, recs, models_info,
             symmetric_ids, batch_fn=None, planned=None):
  """errors dict per record. The gated-in tuples of the scene are evaluated as
  one GPU batch; under torch.distributed (world > 1) the scene's images are
  split over the ranks (LPT on the estimated tuple costs) and the rows gathered
  to rank 0 (RCCL), which alone returns the errors (None elsewhere). planned:
  (errs, todo, mine, depths) prepared ahead by run() (depths: the frames of
  this rank's images, or None), else computed here."""
  et = p["error_type"]
  rank, world = _dist()
  if planned is None:
    objects = getattr(ev, "objects", None)
    planned = plan_rank(p, recs, models_info, objects, scene_camera, dp_split["im_size"], rank,
                        world) + (None,)
  errs, todo, mine, depths = planned
  if todo:
    batch_fn = batch_fn or evaluate_batch
    kw = {"depths": depths} if depths is not None else {}
    if world == 1:
      rows = batch_fn(ev, torch, p, dataset, dp_split, scene_camera, scene_id, recs,
                      models_info, symmetric_ids, todo, **kw)
    else:
      from . import shard
      local = batch_fn(ev, torch, p, dataset, dp_split, scene_camera, scene_id, recs,
                       models_info, symmetric_ids, [todo[i] for i in mine],
                       **kw) if len(mine) else None
      width = len(p["vsd_taus"]) if et == "vsd" else (10 if et == "cus" else 1)
      dev = ev.device if ev is not None else torch.device("cpu")
      if local is None:
        local = torch.zeros((0, width), dtype=torch.float64, device=dev)
      rows = shard.gather_rows(local, torch.as_tensor(mine, dtype=torch.int64, device=dev),
                               len(todo))
  if rank != 0:
    return None
  if todo:
    for (ri, gt_id, _, _), row in zip(todo, rows.cpu().numpy()):
      errs[ri][gt_id] = row_to_errors(et, row)
  return errs


# ------------------------------------------------------------------------ main
def run(p, device=0):
  """Evaluate every result file of p; returns the written file paths."""
  import torch

  if p["error_type"] not in ERROR_TYPES:
    raise ValueError("Unknown pose error function.")
  written = []
  ev = None
  for result_filename in p["result_filenames"]:
    log("Processing: {}".format(result_filename))
    time_start = time.time()
    result_name = os.path.splitext(os.path.basename(result_filename))[0]
    info = result_name.split("_")
    method = str(info[0])
    ds = info[1].split("-")
    dataset, split = str(ds[0]), str(ds[1])
    split_type = str(ds[2]) if len(ds) > 2 else None
    split_type_str = " - " + split_type if split_type is not None else ""
    dp_split = dataset_params.get_split_params(p["datasets_path"], dataset, split, split_type)
    dp_model = dataset_params.get_model_params(p["datasets_path"], dataset, "eval")
    et = p["error_type"]
    # VSD test depth: every target image of every scene, decoded on the GPU in
    # shared launches (depth_gpu.GroupPrefetch) from here on, so the decode
    # overlaps the model upload, the results parse and the planning below
    rank, world = _dist()
    if et not in ("re", "te", "rete") and ev is None:
      ev = evaluator(device)
    up = None
    if et == "vsd" and ev is not None and torch.cuda.is_available():
      # (the prepare thread's uploads and the decoder run on this stream, the
      # main stream only ever sees frames already resident)
      up = (torch.cuda.Stream(ev.device), torch.cuda.current_stream(ev.device))
    arrays = (et in ARRAY_TYPES and world == 1 and ev is not None and
              os.environ.get("BOPX_ERRORS_ARRAYS", "1") != "0")
    groups, group_ims = None, {}
    if arrays and et == "vsd" and up is not None and depth_gpu.enabled() and depth_group_frames() > 0:
      targets = cached_load(inout.load_json,
                            os.path.join(dp_split["base_path"], p["targets_filename"]))
      scene_ims = {}  # scenes in the order organize() gives them, images sorted
      for t in targets:
        scene_ims.setdefault(t["scene_id"], set()).add(t["im_id"])

      def scene_images(scene_id, ims):
        scene_camera = cached_load(inout.load_scene_camera,
                                   dp_split["scene_camera_tpath"].format(scene_id=scene_id))
        group_ims[scene_id] = ims
        return scene_depth_paths(dp_split, scene_camera, scene_id, ims)
      W_, H_ = dp_split["im_size"]
      groups = depth_gpu.GroupPrefetch(
          ev.device.index or 0,
          [(sid, (lambda sid=sid, ims=sorted(v): scene_images(sid, ims)))
           for sid, v in scene_ims.items()],
          H_, W_, torch, up[0], up[1], max_frames=depth_group_sizes()[0],
          first_frames=depth_group_sizes()[1], max_groups=3)
    try:
      models_info = None
      if et in ("ad", "add", "adi", "vsd", "mssd", "mspd", "cus"):
        models_info = cached_load(inout.load_json, dp_model["models_info_path"], keys_to_int=True)
      if et not in ("re", "te", "rete"):
        log("Loading object models...")
        Models(ev, p, dp_model, models_info)
      targets = cached_load(inout.load_json, os.path.join(dp_split["base_path"], p["targets_filename"]))
      log("Loading pose estimates...")
      ests = cached_load(inout.load_bop_results, os.path.join(p["results_path"], result_filename))
      targets_org, ests_org = organize(targets, ests)
      sym_ids = set(dp_model["symmetric_obj_ids"] or [])
      ests_counter = 0

      decoder = [None]  # depth_gpu.DepthDecoder, used by the prefetch thread only

      def prefetch_depths(ims, scene_id, scene_camera):
        # the scene's test depth, resident on the device when the GPU runs the
        # VSD: PNGs decoded by kern_png.hip (depth_gpu; BOPX_DEPTH_GPU=0: host
        # decoder + one upload), on the upload stream
        if up is not None and depth_gpu.enabled():
          paths, scales = scene_depth_paths(dp_split, scene_camera, scene_id, ims)
          W, H = dp_split["im_size"]
          if decoder[0] is None:
            decoder[0] = depth_gpu.DepthDecoder(ev.device.index or 0)
          try:
            with torch.cuda.stream(up[0]):
              d = decoder[0].load(paths, scales, H, W, torch)
            d.record_stream(up[1])  # freed behind the main stream's use
            return d
          except ValueError:
            pass  # a frame of another size: the host path below
        depths = load_scene_depths(dp_split, scene_camera, scene_id, ims, torch,
                                   reuse=up is not None)
        if up is not None and torch.is_tensor(depths):
          with torch.cuda.stream(up[0]):
            d = depths.to(ev.device, non_blocking=True)
          up[0].synchronize()
          d.record_stream(up[1])  # freed behind the main stream's use
          depths = d
        return depths

      scenes = list(targets_org.items())

      def prepare(scene_id, scene_targets):
        # host side of one scene: annotations, records, gates, this rank's share
        # of the tuples and (VSD) its test-depth PNGs, decoded while the previous
        # scene runs and is saved
        scene_camera = cached_load(inout.load_scene_camera,
                                   dp_split["scene_camera_tpath"].format(scene_id=scene_id))
        gt_path = dp_split["scene_gt_tpath"].format(scene_id=scene_id)
        planned = None
        if arrays:
          # the instance lists as arrays, read natively off the GIL (the main
          # thread launches and saves the previous scene meanwhile)
          scene_gt = scene_gt_arrays(gt_path)
          arr, n_ests = scene_arrays_direct_cached(p, scene_id, scene_targets, ests_org, scene_gt)
          recs = None
          vals, todo = plan_arrays(p, arr, models_info)
          depths = depth_ims = None
          if et == "vsd" and not len(todo) and groups is not None:
            release_group_slice(groups, scene_id)
          if et == "vsd" and len(todo):
            if groups is not None:
              try:
                depths = groups.get(scene_id)
                depth_ims = group_ims.get(scene_id)
              except ValueError:
                depths = None  # a frame of another size in the group: per-scene path
            if depths is None:
              depth_ims = None
              depths = prefetch_depths(
                  np.unique(arr["rec_im"][arr["pair_ri"][todo]]).tolist(), scene_id, scene_camera)
          planned = ("arrays", arr, vals, todo, (depths, depth_ims))
          return scene_camera, recs, n_ests, planned
        scene_gt = cached_load(inout.load_scene_gt, gt_path)
        recs, n_ests = scene_records_cached(p, scene_id, scene_targets, ests_org, scene_gt)
        if recs:
          errs, todo, mine = plan_rank(p, recs, models_info, ev.objects if ev else None,
                                       scene_camera, dp_split["im_size"], rank, world)
          depths = None
          if et == "vsd" and len(mine):
            depths = prefetch_depths(todo_images(recs, [todo[i] for i in mine]), scene_id,
                                     scene_camera)
          planned = (errs, todo, mine, depths)
        return scene_camera, recs, n_ests, planned

      from concurrent.futures import ThreadPoolExecutor
      with ThreadPoolExecutor(1) as ahead:
        nxt = ahead.submit(prepare, *scenes[0]) if scenes else None
        for k, (scene_id, scene_targets) in enumerate(scenes):
          scene_camera, recs, n_ests, planned = nxt.result()
          if k + 1 < len(scenes):
            nxt = ahead.submit(prepare, *scenes[k + 1])
          log("Calculating error {} - method: {}, dataset: {}{}, scene: {}".format(
              et, method, dataset, split_type_str, scene_id))
          ests_counter += n_ests
          if arrays:
            _, arr, vals, todo, (depths, depth_ims) = planned
            if len(todo):
              rows = evaluate_batch_arrays(ev, torch, p, dataset, dp_split, scene_camera,
                                           scene_id, arr, todo, models_info, depths, depth_ims)
              vals[todo] = rows.cpu().numpy()
            if et == "vsd":  # one file per tau (:401-415)
              signs = [misc.get_error_signature(et, p["n_top"], vsd_delta=p["vsd_deltas"][dataset],
                                                vsd_tau=tau) for tau in p["vsd_taus"]]
            else:
              signs = [misc.get_error_signature(et, p["n_top"])]
            paths = [p["out_errors_tpath"].format(eval_path=p["eval_path"], result_name=result_name,
                                                  error_sign=sg, scene_id=scene_id) for sg in signs]
            for path in paths:
              os.makedirs(os.path.dirname(path), exist_ok=True)
              log("Saving errors to: {}".format(path))
            inout.save_errors_arrays(paths, arr["rec_im"], arr["rec_obj"], arr["rec_est"],
                                     arr["rec_score"], arr["pair_off"], arr["pair_gt"], vals)
            written.extend(paths)
            continue
          errs = evaluate(ev, torch, p, dataset, dp_split, scene_camera, scene_id, recs,
                          models_info, sym_ids, planned=planned) if recs else []
          if errs is None or _dist()[0] != 0:  # rank 0 writes (also for a scene with no records)
            continue
          scene_errs = [{"im_id": r["im_id"], "obj_id": r["obj_id"], "est_id": r["est_id"],
                         "score": r["score"], "errors": e} for r, e in zip(recs, errs)]

          def save(sign, content):
            path = p["out_errors_tpath"].format(eval_path=p["eval_path"], result_name=result_name,
                                               error_sign=sign, scene_id=scene_id)
            os.makedirs(os.path.dirname(path), exist_ok=True)
            log("Saving errors to: {}".format(path))
            inout.save_json(path, content)
            written.append(path)

          if et == "vsd":
            # one file per tau (:401-415), all written from one encoding per record
            paths = []
            for tau in p["vsd_taus"]:
              sign = misc.get_error_signature(et, p["n_top"], vsd_delta=p["vsd_deltas"][dataset],
                                              vsd_tau=tau)
              paths.append(p["out_errors_tpath"].format(eval_path=p["eval_path"],
                                                        result_name=result_name, error_sign=sign,
                                                        scene_id=scene_id))
              os.makedirs(os.path.dirname(paths[-1]), exist_ok=True)
              log("Saving errors to: {}".format(paths[-1]))
            inout.save_json_per_value(paths, scene_errs, len(paths))
            written.extend(paths)
          else:
            save(misc.get_error_signature(et, p["n_top"]), scene_errs)
    finally:
      if groups is not None:
        groups.close()
    log("Calculation of errors for {} estimates took {}s.".format(
        ests_counter, time.time() - time_start))
  log("Done.")
  return written


def main(argv=None):
  p = parse_args(argv)
  log("-----------")
  log("Parameters:")
  for k, v in p.items():
    log("- {}: {}".format(k, v))
  log("-----------")
  from . import shard
  _, _, local = shard.init_from_env()  # torchrun: scenes' images split over the GPUs
  run(p, local)


if __name__ == "__main__":
  main()
