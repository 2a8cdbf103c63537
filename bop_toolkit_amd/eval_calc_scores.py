"""Counterpart of scripts/eval_calc_scores.py: match the
estimates of every scene to the valid GT poses and compute the localization
recall, from the errors_*.json written by eval_calc_errors.

Same parameters, command line, GT validity rules (visib_gt_min >= 0: visible
fraction threshold; -1: the inst_count most visible GT instances of every
target object, eval_calc_scores.py:183-214), error normalisation (by object
diameter for ad/add/adi/mssd, by 640 / image width for mspd, :221-233) and
output files (matches_{sign}.json, scores_{sign}.json). Host-only: matching
and counting are small integer bookkeeping.

`score_error_dir` is the in-process entry point (eval_bop19_pose calls it for
every threshold without spawning interpreters).
"""
import argparse
import copy
import os
import time

from . import dataset_params, inout, misc, pose_matching, score

DEFAULTS = {
    "correct_th": {"vsd": [0.3], "mssd": [0.2], "mspd": [10], "cus": [0.5], "rete": [5.0, 5.0],
                   "re": [5.0], "te": [5.0], "proj": [5.0], "ad": [0.1], "add": [0.1],
                   "adi": [0.1]},
    "normalized_by_diameter": ["ad", "add", "adi", "mssd"],
    "normalized_by_im_width": ["mspd"],
    "visib_gt_min": -1,
    "error_dir_paths": ["/path/to/calculated/errors"],
    "eval_path": "/path/to/eval/folder",
    "datasets_path": None,  # config.py: $BOP_PATH, read when the arguments are parsed
    "targets_filename": "test_targets_bop19.json",
    "error_tpath": os.path.join("{eval_path}", "{error_dir_path}", "errors_{scene_id:06d}.json"),
    "out_matches_tpath": os.path.join("{eval_path}", "{error_dir_path}",
                                      "matches_{score_sign}.json"),
    "out_scores_tpath": os.path.join("{eval_path}", "{error_dir_path}",
                                     "scores_{score_sign}.json"),
}


def parse_args(argv=None):
  p = copy.deepcopy(DEFAULTS)
  p["datasets_path"] = os.environ.get("BOP_PATH", "/path/to/bop/datasets")
  ap = argparse.ArgumentParser()
  for et, th in p["correct_th"].items():
    ap.add_argument("--correct_th_" + et, default=",".join(map(str, th)))
  ap.add_argument("--normalized_by_diameter", default=",".join(p["normalized_by_diameter"]))
  ap.add_argument("--normalized_by_im_width", default=",".join(p["normalized_by_im_width"]))
  ap.add_argument("--visib_gt_min", default=p["visib_gt_min"])
  ap.add_argument("--error_dir_paths", default=",".join(p["error_dir_paths"]))
  for k in ("eval_path", "datasets_path", "targets_filename", "error_tpath",
            "out_matches_tpath", "out_scores_tpath"):
    ap.add_argument("--" + k, default=p[k])
  a = ap.parse_args(argv)
  for et in p["correct_th"]:
    p["correct_th"][et] = [float(x) for x in getattr(a, "correct_th_" + et).split(",")]
  p["normalized_by_diameter"] = a.normalized_by_diameter.split(",")
  p["normalized_by_im_width"] = a.normalized_by_im_width.split(",")
  p["visib_gt_min"] = float(a.visib_gt_min)
  p["error_dir_paths"] = a.error_dir_paths.split(",")
  for k in ("eval_path", "datasets_path", "targets_filename", "error_tpath",
            "out_matches_tpath", "out_scores_tpath"):
    p[k] = str(getattr(a, k))
  return p


def valid_gts(im_gt, im_gt_info, im_targets, visib_gt_min):
  """Which GT instances of an image count (eval_calc_scores.py:183-214)."""
  if visib_gt_min >= 0:
    return [gt["obj_id"] in im_targets and im_gt_info[g]["visib_fract"] >= visib_gt_min
            for g, gt in enumerate(im_gt)]
  valid = [False] * len(im_gt)
  left = {o: t["inst_count"] for o, t in im_targets.items()}
  for g in sorted(range(len(im_gt)), key=lambda g: im_gt_info[g]["visib_fract"], reverse=True):
    o = im_gt[g]["obj_id"]
    if left.get(o, 0) > 0:
      valid[g] = True
      left[o] -= 1
  return valid


class _Cache:
  """Per-dataset inputs shared by all thresholds of one evaluation, and the
  parsed (normalised, grouped) errors files of the most recent errors folder:
  eval_bop19_pose scores every folder at 10 thresholds in a row."""

  def __init__(self):
    import threading
    self.d = {}
    self._folder = None
    self._errs = {}
    self._lock = threading.RLock()  # FolderScorer's threads share one cache

  def get(self, key, fn):
    with self._lock:
      if key not in self.d:
        self.d[key] = fn()
      return self.d[key]

  def errors(self, folder, path, fn):
    if folder != self._folder:
      self._folder, self._errs = folder, {}
    st = os.stat(path)
    key = (path, st.st_mtime_ns, st.st_size)
    if key not in self._errs:
      self._errs[key] = fn()
    return self._errs[key]


def _load_errors(path, models_info, by_dia, width_factor):
  """errors_*.json of a scene, normalised (eval_calc_scores.py:221-233) and
  grouped per (image, object) in match order."""
  scene_errs = inout.load_json(path, keys_to_int=True)
  if by_dia:
    for err in scene_errs:
      dia = float(models_info[err["obj_id"]]["diameter"])
      err["errors"] = {g: [e / dia for e in v] for g, v in err["errors"].items()}
  if width_factor is not None:
    for err in scene_errs:
      err["errors"] = {g: [width_factor * e for e in v] for g, v in err["errors"].items()}
  return pose_matching.group_scene_errs(scene_errs)


def score_error_dir(p, error_dir_path, correct_th=None, cache=None, do_print=True):
  """Matches + scores of one errors folder; returns (scores, score_sign)."""
  cache = cache or _Cache()
  error_sign = os.path.basename(error_dir_path)
  err_type = str(error_sign.split("_")[0].split("=")[1])
  n_top = int(error_sign.split("_")[1].split("=")[1])
  info = os.path.basename(os.path.dirname(error_dir_path)).split("_")
  method, ds = info[0], info[1].split("-")
  dataset, split = ds[0], ds[1]
  split_type = ds[2] if len(ds) > 2 else None
  th = p["correct_th"][err_type] if correct_th is None else correct_th
  score_sign = misc.get_score_signature(th, p["visib_gt_min"])
  misc.log("Calculating score - error: {}, method: {}, dataset: {}.".format(
      err_type, method, dataset))
  dp_split = dataset_params.get_split_params(p["datasets_path"], dataset, split, split_type)
  dp_model = dataset_params.get_model_params(p["datasets_path"], dataset, "eval")
  models_info = cache.get(("info", dp_model["models_info_path"]), lambda: inout.load_json(
      dp_model["models_info_path"], keys_to_int=True))
  tpath = os.path.join(dp_split["base_path"], p["targets_filename"])
  targets = cache.get(("targets", tpath), lambda: inout.load_json(tpath))
  targets_org = {}
  for t in targets:
    targets_org.setdefault(t["scene_id"], {}).setdefault(t["im_id"], {})[t["obj_id"]] = t
  matches = []
  for scene_id, scene_targets in targets_org.items():
    gpath = dp_split["scene_gt_tpath"].format(scene_id=scene_id)
    scene_gt = cache.get(("gt", gpath), lambda: inout.load_scene_gt(gpath))
    ipath = dp_split["scene_gt_info_tpath"].format(scene_id=scene_id)
    scene_gt_info = cache.get(("gti", ipath), lambda: inout.load_json(ipath, keys_to_int=True))
    gt_curr = {im: scene_gt[im] for im in scene_targets}
    gt_valid = cache.get(("valid", ipath, tpath, p["visib_gt_min"]), lambda: {
        im: valid_gts(scene_gt[im], scene_gt_info[im], tg, p["visib_gt_min"])
        for im, tg in scene_targets.items()})
    epath = p["error_tpath"].format(eval_path=p["eval_path"], error_dir_path=error_dir_path,
                                    scene_id=scene_id)
    by_dia = err_type in p["normalized_by_diameter"]
    factor = (640.0 / float(dp_split["im_size"][0])
              if err_type in p["normalized_by_im_width"] else None)
    scene_errs = cache.errors(error_dir_path, epath,
                              lambda: _load_errors(epath, models_info, by_dia, factor))
    matches += pose_matching.match_poses_scene(scene_id, gt_curr, gt_valid, scene_errs, th,
                                               n_top)
  scores = score.calc_localization_scores(dp_split["scene_ids"], dp_model["obj_ids"], matches,
                                          n_top, do_print=do_print)
  fmt = dict(eval_path=p["eval_path"], error_dir_path=error_dir_path, score_sign=score_sign)
  inout.save_json(p["out_scores_tpath"].format(**fmt), scores)
  inout.save_json(p["out_matches_tpath"].format(**fmt), matches)
  return scores, score_sign


def _score_job(job):
  error_dir_path, sps, do_print = job
  cache = _Cache()
  if os.environ.get("BOPX_SCORE_NATIVE", "1") != "0":
    out = score_error_dir_native(sps, error_dir_path, cache=cache, do_print=do_print)
    if out is not None:
      return [sc for sc, _ in out]
  return [score_error_dir(sp, error_dir_path, cache=cache, do_print=do_print)[0] for sp in sps]


_SCORE_LIB = None


def _score_lib():
  """ctypes handle of bopx_score_folder (include/bopx_score.h) in libbopx_io.so."""
  global _SCORE_LIB
  if _SCORE_LIB is None:
    import ctypes as C

    class Args(C.Structure):
      _fields_ = [("n_gt", C.c_int64), ("gt_scene", C.c_void_p), ("gt_im", C.c_void_p),
                  ("gt_obj", C.c_void_p), ("gt_id", C.c_void_p), ("gt_valid", C.c_void_p),
                  ("n_im", C.c_int64), ("im_off", C.c_void_p), ("im_file", C.c_void_p),
                  ("n_files", C.c_int), ("err_paths", C.POINTER(C.c_char_p)),
                  ("norm", C.c_int), ("n_diam", C.c_int), ("diam", C.c_void_p),
                  ("width_factor", C.c_double), ("n_top", C.c_int), ("n_settings", C.c_int),
                  ("n_th", C.c_int), ("th", C.c_void_p), ("matches_paths", C.POINTER(C.c_char_p)),
                  ("matched", C.c_void_p), ("threads", C.c_int)]
    lib = inout._io_lib()
    lib.bopx_score_folder.argtypes = [C.POINTER(Args), C.c_char_p, C.c_int]
    lib.bopx_score_folder.restype = C.c_int
    _SCORE_LIB = (lib, Args)
  return _SCORE_LIB


# Dataset side of the native scorer, kept for the process (like the error
# passes' file cache): the targets' organised view, the GT table and its
# ArrayScorer, keyed on the identities of the parsed files they come from
# (eval_calc_errors.cached_load returns a new object when a file changes), so
# a second evaluation in the process does not rebuild them in Python while
# its error passes run (the GIL).
_DS_CACHE = {}
_DS_LOCK = None


def _ds_cached(key, keep, fn):
  """fn() cached under key; keep: the objects whose id() is in the key (held
  with the value so the ids stay theirs)."""
  import threading
  global _DS_LOCK
  if _DS_LOCK is None:
    _DS_LOCK = threading.RLock()
  with _DS_LOCK:
    hit = _DS_CACHE.get(key)
    if hit is None:
      if len(_DS_CACHE) > 32:
        _DS_CACHE.clear()
      with inout.gc_paused():  # bulk acyclic builds (the GT table, the targets' view)
        hit = _DS_CACHE[key] = (keep, fn())
    return hit[1]


def _gt_table(cache, dp_split, targets_org, visib_gt_min):
  """The matches file's GT records in order (targets' scenes and images, every
  GT of an image) as arrays, with per-image offsets and scene index
  (score_error_dir's scene_gt / gt_valid, eval_calc_scores.py:183-214)."""
  import numpy as np
  from .eval_calc_errors import cached_load, scene_gt_arrays  # the error passes' parses
  gts = []
  for scene_id in targets_org:
    # the native readers' arrays (no Python JSON parse under the GIL while the
    # next error pass runs), or the dicts when either file is declined
    gpath = dp_split["scene_gt_tpath"].format(scene_id=scene_id)
    ipath = dp_split["scene_gt_info_tpath"].format(scene_id=scene_id)
    g = scene_gt_arrays(gpath)
    i = cached_load(inout.load_scene_gt_info_lists, ipath) if isinstance(g, inout.GTLists) \
        else None
    if i is None:
      g = cached_load(inout.load_scene_gt, gpath)
      i = cached_load(inout.load_json, ipath, keys_to_int=True)
    gts.append((g, i))

  def lists_image(scene_gt, scene_gt_info, im_id):
    # (obj ids, [{"visib_fract"}]) of an image, as valid_gts reads the dicts;
    # an info list shorter than the GT list indexes past its end there too
    a, b = scene_gt.rows(im_id)
    c, d = scene_gt_info.rows(im_id)
    vf = scene_gt_info.fields["visib_fract"][c:d, 0].tolist()
    return [{"obj_id": o} for o in scene_gt.obj[a:b].tolist()], [{"visib_fract": v} for v in vf]

  def build():
    sc, im, ob, gid, val, off, fi = [], [], [], [], [], [0], []
    for k, (scene_id, scene_targets) in enumerate(targets_org.items()):
      scene_gt, scene_gt_info = gts[k]
      lists = isinstance(scene_gt, inout.GTLists)
      for im_id, tg in scene_targets.items():
        if lists:
          im_gts, im_info = lists_image(scene_gt, scene_gt_info, im_id)
        else:
          im_gts, im_info = scene_gt[im_id], scene_gt_info[im_id]
        valid = valid_gts(im_gts, im_info, tg, visib_gt_min)
        for g, gt in enumerate(im_gts):
          sc.append(scene_id)
          im.append(im_id)
          ob.append(gt["obj_id"])
          gid.append(g)
          val.append(bool(valid[g]))
        off.append(len(sc))
        fi.append(k)
    i32 = lambda a: np.ascontiguousarray(a, np.int32)
    return (i32(sc), i32(im), i32(ob), i32(gid), np.ascontiguousarray(val, np.uint8),
            np.ascontiguousarray(off, np.int64), i32(fi))
  key = ("gt_table", dp_split["base_path"], id(targets_org), visib_gt_min,
         tuple((id(a), id(b)) for a, b in gts))
  return _ds_cached(key, (targets_org, gts), build)


def score_error_dir_native(sps, error_dir_path, cache=None, do_print=True, threads=0):
  """score_error_dir for every setting in sps (one errors folder; the settings
  differ only in correct_th) through the native scorer (bopx_score_folder:
  the errors files parsed once, the matches files written by C++, the same
  bytes). Returns [(scores, score_sign)] in sps order, or None when the
  scorer declines the inputs (the Python path then runs and raises what the
  reference raises)."""
  import ctypes as C

  import numpy as np
  if not sps:
    return []
  p = sps[0]
  cache = cache or _Cache()
  error_sign = os.path.basename(error_dir_path)
  err_type = str(error_sign.split("_")[0].split("=")[1])
  n_top = int(error_sign.split("_")[1].split("=")[1])
  for sp in sps[1:]:
    if any(sp[k] != p[k] for k in p if k != "correct_th"):
      return None
  ths = [sp["correct_th"][err_type] for sp in sps]
  if len(set(len(t) for t in ths)) != 1:
    return None
  info = os.path.basename(os.path.dirname(error_dir_path)).split("_")
  method, ds = info[0], info[1].split("-")
  dataset, split = ds[0], ds[1]
  split_type = ds[2] if len(ds) > 2 else None
  dp_split = dataset_params.get_split_params(p["datasets_path"], dataset, split, split_type)
  dp_model = dataset_params.get_model_params(p["datasets_path"], dataset, "eval")
  from .eval_calc_errors import cached_load  # the error passes' parses (same process)
  models_info = cached_load(inout.load_json, dp_model["models_info_path"], keys_to_int=True)
  tpath = os.path.join(dp_split["base_path"], p["targets_filename"])
  targets = cached_load(inout.load_json, tpath)

  def org():
    t_org = {}
    for t in targets:
      t_org.setdefault(t["scene_id"], {}).setdefault(t["im_id"], {})[t["obj_id"]] = t
    return t_org
  targets_org = _ds_cached(("targets_org", id(targets)), targets, org)
  sc, im, ob, gid, val, off, fi = _gt_table(cache, dp_split, targets_org, p["visib_gt_min"])
  err_paths = [p["error_tpath"].format(eval_path=p["eval_path"], error_dir_path=error_dir_path,
                                       scene_id=scene_id) for scene_id in targets_org]
  signs = [misc.get_score_signature(th, p["visib_gt_min"]) for th in ths]
  mpaths = [p["out_matches_tpath"].format(eval_path=p["eval_path"], error_dir_path=error_dir_path,
                                          score_sign=sg) for sg in signs]
  lib, Args = _score_lib()
  norm, diam, factor = 0, np.zeros(1), 0.0
  if err_type in p["normalized_by_diameter"]:
    ids = [o for o in models_info if isinstance(o, int) and o >= 0]
    if not ids or len(ids) != len(models_info):
      return None
    diam = np.full(max(ids) + 1, np.nan)
    for o in ids:
      diam[o] = float(models_info[o]["diameter"])
    norm = 1
  elif err_type in p["normalized_by_im_width"]:
    norm, factor = 2, 640.0 / float(dp_split["im_size"][0])
  th = np.ascontiguousarray(ths, np.float64)
  matched = np.zeros((len(sps), len(sc)), np.uint8)
  paths_c = (C.c_char_p * len(err_paths))(*[x.encode() for x in err_paths])
  mpaths_c = (C.c_char_p * len(mpaths))(*[x.encode() for x in mpaths])
  diam = np.ascontiguousarray(diam, np.float64)
  ptr = lambda a: a.ctypes.data
  a = Args(len(sc), ptr(sc), ptr(im), ptr(ob), ptr(gid), ptr(val), len(off) - 1, ptr(off),
           ptr(fi), len(err_paths), paths_c, norm, len(diam), ptr(diam), factor, n_top,
           len(sps), th.shape[1], ptr(th), mpaths_c, ptr(matched),
           int(os.environ.get("BOPX_SCORE_THREADS", "0")) or threads or min(len(sps), 8))
  for sg in signs:
    misc.log("Calculating score - error: {}, method: {}, dataset: {}.".format(
        err_type, method, dataset))
  msg = C.create_string_buffer(512)
  st = lib.bopx_score_folder(C.byref(a), msg, len(msg))
  if st in (1, 2, 3):
    # unreadable / unparsable errors files or inputs the scorer does not take
    # (BOPX_SCORE_READ, _PARSE, _UNSUPPORTED): the Python path, which raises
    # what the reference raises for bad files
    return None
  if st != 0:
    raise RuntimeError("bopx_score_folder: %s (status %d)" % (msg.value.decode(), st))
  scorer = _ds_cached(("scorer", id(sc), n_top, tuple(dp_split["scene_ids"]),
                      tuple(dp_model["obj_ids"])), sc, lambda: score.ArrayScorer(
      dp_split["scene_ids"], dp_model["obj_ids"], sc, im, ob, val, n_top))
  out = []
  for k, sg in enumerate(signs):
    scores = scorer.scores(matched[k], do_print=do_print)
    fmt = dict(eval_path=p["eval_path"], error_dir_path=error_dir_path, score_sign=sg)
    inout.save_json(p["out_scores_tpath"].format(**fmt), scores)
    out.append((scores, sg))
  return out


def _lower_priority():
  try:
    os.nice(5)
  except OSError:
    pass


def _score_job_threaded(job, cache, threads):
  """_score_job in a thread of the calling process (native scorer: the GIL is
  released while it runs; the GT side is parsed once for all folders)."""
  error_dir_path, sps, do_print = job
  out = score_error_dir_native(sps, error_dir_path, cache=cache, do_print=do_print,
                               threads=threads)
  if out is not None:
    return [sc for sc, _ in out]
  own = _Cache()  # the Python path (inputs the native scorer declines)
  return [score_error_dir(sp, error_dir_path, cache=own, do_print=do_print)[0] for sp in sps]


def _native_available():
  if os.environ.get("BOPX_SCORE_NATIVE", "1") == "0":
    return False
  try:
    _score_lib()
    return True
  except (OSError, AttributeError, RuntimeError):
    return False


class FolderScorer:
  """score_folders in stages: submit(jobs) queues a group of folders (scored
  at once while the caller goes on, e.g. computes the next error type's
  folders on the GPU), results() returns every group's scores in submission
  order.

  Native scorer (libbopx_io.so, the default): a pool of threads of this
  process, each folder one bopx_score_folder call over all its settings, the
  GT side parsed once (shared with the error passes' file cache). Without it
  (BOPX_SCORE_NATIVE=0): a pool of spawned processes running the Python
  scorer, started at once at a lower CPU priority (nice +5), so their
  interpreter start-up runs behind the caller's first error pass
  (BOPX_SCORE_EARLY=0: start with the first submit)."""

  def __init__(self, n_folders, workers=None, do_print=True):
    self.native = _native_available()
    if workers is None:
      workers = int(os.environ.get("BOPX_SCORE_WORKERS", "0")) or \
          min(n_folders, os.cpu_count() or 1, 8 if self.native else 16)
    self.do_print = do_print
    self.workers = workers if n_folders > 1 else 1
    self.pool = None
    self.tpool = None
    self.cache = _Cache()
    self.pending = []
    if self.native:
      from concurrent.futures import ThreadPoolExecutor
      self.tpool = ThreadPoolExecutor(max(1, self.workers))
    elif self.workers > 1 and os.environ.get("BOPX_SCORE_EARLY", "1") != "0":
      self._start()

  def _start(self):
    import multiprocessing as mp
    self.pool = mp.get_context("spawn").Pool(self.workers, initializer=_lower_priority)

  def submit(self, jobs):
    args = [(path, sps, self.do_print) for path, sps in jobs]
    if self.tpool is not None:
      # native threads per folder: the host's scoring share (16) over the group
      thr = max(1, 16 // max(1, len(args)))
      self.pending.append([[self.tpool.submit(_score_job_threaded, a, self.cache, thr)]
                           for a in args])
      return
    if self.pool is None and self.workers > 1:
      self._start()
    if self.pool is None:
      self.pending.append([[_score_job(a)] for a in args])  # one finished chunk per folder
      return
    # A group of fewer folders than workers (MSSD, MSPD: one folder of ten
    # thresholds each) spreads each folder's settings over the idle workers in
    # contiguous chunks; a chunk re-reads the folder's errors, the scores are
    # the same (BOPX_SCORE_SPLIT=0: one task per folder)
    split = os.environ.get("BOPX_SCORE_SPLIT", "1") != "0"
    group = []
    for path, sps, do_print in args:
      k = max(1, min(len(sps), self.workers // max(1, len(args)))) if split else 1
      cut = [len(sps) * i // k for i in range(k + 1)]
      group.append([self.pool.apply_async(_score_job, ((path, sps[cut[i]:cut[i + 1]], do_print),))
                    for i in range(k)])
    self.pending.append(group)

  def results(self):
    try:
      out = []
      for group in self.pending:  # per folder: its chunks' scores in setting order
        for chunks in group:
          got = []
          for c in chunks:
            got += c if isinstance(c, list) else (c.result() if hasattr(c, "result") else c.get())
          out.append(got)
      return out
    finally:
      self.close()

  def close(self):
    """Stops the pools (after results(), or on an error: terminates them)."""
    if self.pool is not None:
      self.pool.terminate()
      self.pool.join()
      self.pool = None
    if self.tpool is not None:
      self.tpool.shutdown(wait=True)
      self.tpool = None


def score_folders(jobs, workers=None, do_print=True):
  """Scores of several errors folders, each at several settings: jobs is a
  list of (error_dir_path, [params per setting]); returns the scores dicts in
  the same nesting and order. Folders are independent (the reference scores
  every setting in its own interpreter, eval_bop19_pose.py:150-213), so with
  more than one worker they are scored in a pool of spawned processes
  (host-only modules: no GPU state is inherited). workers: default
  $BOPX_SCORE_WORKERS, else min(#folders, CPUs, 16)."""
  if workers is None:
    workers = int(os.environ.get("BOPX_SCORE_WORKERS", "0")) or \
        min(len(jobs), os.cpu_count() or 1, 16)
  args = [(path, sps, do_print) for path, sps in jobs]
  if workers <= 1 or len(jobs) <= 1:
    return [_score_job(a) for a in args]
  import multiprocessing as mp
  with mp.get_context("spawn").Pool(workers) as pool:
    return pool.map(_score_job, args, chunksize=1)


def main(argv=None):
  p = parse_args(argv)
  misc.log("-----------")
  misc.log("Parameters:")
  for k, v in p.items():
    misc.log("- {}: {}".format(k, v))
  misc.log("-----------")
  for error_dir_path in p["error_dir_paths"]:
    misc.log("Processing: {}".format(error_dir_path))
    t0 = time.time()
    score_error_dir(p, error_dir_path)
    misc.log("Matching and score calculation took {}s.".format(time.time() - t0))
  misc.log("Done.")


if __name__ == "__main__":
  main()
