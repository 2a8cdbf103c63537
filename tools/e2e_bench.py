#!/usr/bin/env python
"""End-to-end timing of the BOP19 evaluation pipeline on a synthetic dataset.

Writes a YCB-V-layout dataset (21 superellipsoid objects of 5,002 vertices,
test scenes 48.., 6 objects per image, 16-bit depth PNGs with depth_scale 0.1
rendered by the HIP rasteriser plus background, occluder, noise and holes) and
a BOP19 results CSV, then times the drop-in pipeline as a user runs it:

  1. calc_gt_info (scene_gt_info.json; gt_side.calc_gt_info),
  2. eval_bop19_pose: VSD / MSSD / MSPD error files (eval_calc_errors.run)
     and the 120 score settings (eval_calc_scores.score_error_dir),

and prints one JSON line with the per-phase wall times and the end-to-end
tuples/s. --profile adds a cProfile of phase 2 (host hot spots) to
gpurun_out/e2e_profile.txt. Needs a GPU.

    python tools/e2e_bench.py --images 2000 [--root /tmp/bopx_e2e] [--profile]
"""
import argparse
import json
import os
import shutil
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

W, H = 640, 480
DEPTH_SCALE = 0.1
PER_IMG = 6
SCENES = list(range(48, 60))


def progress(msg):
  """Progress line on stderr (long generations: the GPU runner wants output)."""
  print("[e2e %.0fs] %s" % (time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)


T_START = time.perf_counter()


def _save_pngs(npy, jobs):
  """Worker process: Pillow-encode the frames of `jobs` ((path, index) pairs)
  from the memory-mapped uint16 array `npy` (Pillow's encoder holds the GIL,
  so threads do not scale)."""
  from PIL import Image
  arr = np.load(npy, mmap_mode="r")
  for path, i in jobs:
    Image.fromarray(np.ascontiguousarray(arr[i])).save(path)
  return len(jobs)


def write_pngs(root, png, jobs, workers=16):
  """The depth PNGs, Pillow-written by `workers` spawned processes (children
  started with fork + exec, which this GPU-initialised process may do) from
  a memory-mapped copy of the frames; progress every ~1,000 files."""
  import multiprocessing as mp
  from concurrent.futures import ProcessPoolExecutor, as_completed
  npy = os.path.join(root, "frames_u16.npy")
  np.save(npy, png)
  chunk = 256
  parts = [[(p, int(i)) for p, i in jobs[k:k + chunk]] for k in range(0, len(jobs), chunk)]
  done = 0
  try:
    with ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("spawn")) as pool:
      futs = [pool.submit(_save_pngs, npy, part) for part in parts]
      for f in as_completed(futs):
        k = f.result()
        done += k
        if done // 1000 != (done - k) // 1000:
          progress("%d / %d PNGs written" % (done, len(jobs)))
  finally:
    os.remove(npy)


def make_dataset(root, n_im, seed, torch, inst=1):
  from bop_toolkit_amd import inout, misc, synth
  from bop_toolkit_amd.batch import BatchEvaluator
  rng = np.random.default_rng(seed)
  ds = os.path.join(root, "datasets", "ycbv")
  mdir = os.path.join(ds, "models_eval")
  os.makedirs(mdir)
  ev = BatchEvaluator(0)
  info = {}
  for o in range(1, 22):
    axes = tuple(rng.uniform(30.0, 100.0, 3))
    pts, faces = synth.superellipsoid(50, 100, axes, float(rng.uniform(0.5, 1.0)))
    n_disc = [1, 2, 4, 8][o % 4]
    e = synth.models_info_entry(pts, n_disc, continuous=(o == 21))
    info[str(o)] = {k: (float(v) if not isinstance(v, list) else v) for k, v in e.items()}
    inout.save_ply(os.path.join(mdir, "obj_%06d.ply" % o), pts, faces)
    ev.add_object(o, pts.astype(np.float64), faces)
  with open(os.path.join(mdir, "models_info.json"), "w") as f:
    json.dump(info, f)
  shutil.copytree(mdir, os.path.join(ds, "models"))

  # inst > 1 (T-LESS / IC-BIN-like): PER_IMG // 2 objects per image with `inst`
  # instances each and `inst` estimates of each (n_top = -1 pairs all of them)
  per_obj = PER_IMG if inst == 1 else max(1, PER_IMG // 2)
  per_img = per_obj * inst
  obj = np.stack([np.repeat(rng.choice(np.arange(1, 22), per_obj, replace=False), inst)
                  for _ in range(n_im)]).reshape(-1).astype(np.int32)
  n = len(obj)
  Rg, tg = synth.gt_poses(rng, n)
  Re, te = synth.perturb(rng, Rg, tg)
  K = synth.YCBV_K
  dev = ev.device
  T = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
  fidx = np.repeat(np.arange(n_im, dtype=np.int32), per_img)
  cam = np.tile([K[0, 0], K[1, 1], K[0, 2], K[1, 2]], (n_im, 1)).astype(np.float64)
  frames = ev.render(ev.slots(obj), T(np.concatenate([Rg.reshape(n, 9), tg], 1), torch.float64),
                     T(fidx, torch.int32), T(cam, torch.float64), n_im, W, H)
  g = torch.Generator(device=dev)
  g.manual_seed(seed)
  frames = torch.where(frames > 0, frames, torch.full_like(frames, 1600.0))
  ys = torch.arange(H, device=dev).view(1, H, 1)
  xs = torch.arange(W, device=dev).view(1, 1, W)
  x0 = torch.randint(0, W - 120, (n_im, 1, 1), device=dev, generator=g)
  y0 = torch.randint(0, H - 120, (n_im, 1, 1), device=dev, generator=g)
  sz = torch.randint(40, 120, (n_im, 1, 1), device=dev, generator=g)
  occ = (xs >= x0) & (xs < x0 + sz) & (ys >= y0) & (ys < y0 + sz)
  frames = torch.where(occ, torch.full_like(frames, 450.0), frames)
  frames = frames + 2.0 * torch.randn(frames.shape, device=dev, generator=g)
  frames[torch.rand(frames.shape, device=dev, generator=g) < 0.1] = 0.0
  png = torch.round(frames / DEPTH_SCALE).clamp_(0, 65535).to(torch.int32).to(torch.int16)
  png = png.cpu().numpy().view(np.uint16)  # 0..65535 through the int16 bit pattern
  del frames
  progress("rendered %d frames" % n_im)

  scene_of = np.array([SCENES[i * len(SCENES) // n_im] for i in range(n_im)])
  targets, lines = [], ["scene_id,im_id,obj_id,score,R,t,time"]
  jobs = []
  for s in sorted(set(scene_of.tolist())):
    sdir = os.path.join(ds, "test", "%06d" % s)
    os.makedirs(os.path.join(sdir, "depth"))
    cams, gts = {}, {}
    for im in np.nonzero(scene_of == s)[0]:
      jobs.append((os.path.join(sdir, "depth", "%06d.png" % im), im))
      cams[str(im)] = {"cam_K": K.reshape(-1).tolist(), "depth_scale": DEPTH_SCALE}
      rows = range(im * per_img, (im + 1) * per_img)
      gts[str(im)] = [{"cam_R_m2c": Rg[j].reshape(-1).tolist(), "cam_t_m2c": tg[j].tolist(),
                       "obj_id": int(obj[j])} for j in rows]
      for j in rows:
        if j % inst == 0:
          targets.append({"im_id": int(im), "inst_count": inst, "obj_id": int(obj[j]),
                          "scene_id": s})
        lines.append("%d,%d,%d,%r,%s,%s,0.5" % (
            s, im, obj[j], float(rng.random()), " ".join(repr(float(x)) for x in Re[j].ravel()),
            " ".join(repr(float(x)) for x in te[j])))
    with open(os.path.join(sdir, "scene_camera.json"), "w") as f:
      json.dump(cams, f)
    with open(os.path.join(sdir, "scene_gt.json"), "w") as f:
      json.dump(gts, f)
  write_pngs(root, png, jobs)
  del png
  with open(os.path.join(ds, "test_targets_bop19.json"), "w") as f:
    json.dump(targets, f)
  os.makedirs(os.path.join(root, "results"))
  result = "synth_ycbv-test.csv"
  with open(os.path.join(root, "results", result), "w") as f:
    f.write("\n".join(lines) + "\n")
  del ev
  return n * inst, result, sorted(set(scene_of.tolist()))  # tuples: inst^2 per object


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--images", type=int, default=2000)
  ap.add_argument("--root", default="/tmp/bopx_e2e")
  ap.add_argument("--seed", type=int, default=7)
  ap.add_argument("--profile", action="store_true")
  ap.add_argument("--instances", type=int, default=1,
                  help="instances (and estimates) per object and image; > 1: multi-instance")
  ap.add_argument("--ab-group", default=None,
                  help="with --ab-depth: comma list of BOPX_DEPTH_GROUP_FRAMES values (0 = one "
                       "decode launch per scene), each run warm twice, interleaved")
  ap.add_argument("--ab-depth", action="store_true",
                  help="evaluate twice: test depth decoded on the GPU, then on the host "
                       "(BOPX_DEPTH_GPU=0); both timings and identical scores reported")
  ap.add_argument("--warm-reps", type=int, default=2, help="with --ab-group: warm runs per value")
  ap.add_argument("--profile-gt", action="store_true", help="cProfile calc_gt_info")
  a = ap.parse_args()
  import torch
  if os.path.exists(a.root):
    shutil.rmtree(a.root)
  t0 = time.perf_counter()
  n, result, scenes = make_dataset(a.root, a.images, a.seed, torch, a.instances)
  t_gen = time.perf_counter() - t0
  datasets = os.path.join(a.root, "datasets")
  os.environ["BOP_PATH"] = datasets

  from bop_toolkit_amd import eval_bop19_pose, eval_calc_errors as ece, eval_calc_scores as ecs
  from bop_toolkit_amd import gt_side, misc
  misc.log = lambda s: None  # keep stdout to the JSON line
  phases = {}

  def timed(name, fn):
    def wrap(*args, **kw):
      t = time.perf_counter()
      try:
        return fn(*args, **kw)
      finally:
        phases[name] = phases.get(name, 0.0) + time.perf_counter() - t
    return wrap

  gprof = None
  if a.profile_gt:
    import cProfile
    gprof = cProfile.Profile()
    gprof.enable()
  t0 = time.perf_counter()
  gt_side.calc_gt_info({"dataset": "ycbv", "dataset_split": "test", "dataset_split_type": None,
                        "delta": 15, "renderer_type": "hip", "datasets_path": datasets,
                        "scene_ids": scenes})
  torch.cuda.synchronize()
  phases["calc_gt_info"] = time.perf_counter() - t0
  if gprof is not None:
    import io
    import pstats
    gprof.disable()
    s_ = io.StringIO()
    pstats.Stats(gprof, stream=s_).sort_stats("cumulative").print_stats(35)
    pstats.Stats(gprof, stream=s_).sort_stats("tottime").print_stats(25)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "gt_profile.txt"), "w") as f:
      f.write(s_.getvalue())

  # the decoder's counters of calc_gt_info, then zeroed for the evaluation
  from bop_toolkit_amd import depth_gpu as _dg
  gt_stats = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in _dg.STATS.items()}
  for k in _dg.STATS:
    _dg.STATS[k] = 0 if k in ("calls", "frames") else 0.0
  # the evaluation starts cold: nothing calc_gt_info parsed stays in the caches
  ece._FILE_CACHE.clear()
  ece._ORG_CACHE.clear()
  ecs._DS_CACHE.clear()
  run0, score0 = ece.run, ecs.score_error_dir
  err_t = {}

  marks = {}  # wall clock of the last error pass's end; scorer job intervals

  def run_wrap(p, device=0):
    t = time.perf_counter()
    out = run0(p, device)
    err_t[p["error_type"]] = time.perf_counter() - t
    marks["errors_end"] = time.perf_counter()
    return out
  ece.run = run_wrap
  job0 = ecs._score_job_threaded

  def job_wrap(job, cache, threads):
    t = time.perf_counter()
    try:
      return job0(job, cache, threads)
    finally:
      marks.setdefault("jobs", []).append((t, time.perf_counter(), os.path.basename(job[0])))
  ecs._score_job_threaded = job_wrap

  def tail_info(t_end):
    jobs = marks.get("jobs", [])
    return {"after_last_error_pass_s": round(t_end - marks.get("errors_end", t_end), 3),
            "scoring_busy_s": round(sum(b - a for a, b, _ in jobs), 3),
            "scoring_after_errors_s": round(max([b for _, b, _ in jobs] or [0]) -
                                            marks.get("errors_end", 0), 3)}
  ecs.score_error_dir = timed("scores", score0)
  # host steps of the error passes (the prepare thread's included)
  from bop_toolkit_amd import depth_gpu, inout
  depth_gpu.DepthDecoder.load = timed("host:gpu_depth_load", depth_gpu.DepthDecoder.load)
  # timeline of the cold run: (name, start, end) of the host steps on every thread
  tl = []

  def traced(name, fn):
    import functools

    @functools.wraps(fn)
    def wrap(*args, **kw):
      t = time.perf_counter()
      try:
        return fn(*args, **kw)
      finally:
        tl.append((name, t, time.perf_counter()))
    return wrap
  depth_gpu.DepthDecoder.submit = traced("decoder.submit", depth_gpu.DepthDecoder.submit)
  depth_gpu.DepthDecoder.finish = traced("decoder.finish", depth_gpu.DepthDecoder.finish)
  depth_gpu.GroupPrefetch.get = traced("groups.get", depth_gpu.GroupPrefetch.get)
  from bop_toolkit_amd import batch as _batch
  _batch.BatchEvaluator.set_symmetries = traced("ev.set_symmetries",
                                                _batch.BatchEvaluator.set_symmetries)
  _batch.BatchEvaluator.add_object = traced("ev.add_object", _batch.BatchEvaluator.add_object)
  misc.get_symmetry_transformations = traced("get_symmetry_transformations",
                                             misc.get_symmetry_transformations)
  inout.load_bop_results = traced("load_bop_results", inout.load_bop_results)
  for nm in ("organize", "evaluate_batch_arrays", "run", "Models", "plan_arrays",
             "scene_arrays_direct_cached"):
    setattr(ece, nm, traced(nm, getattr(ece, nm)))
  inout.save_errors_arrays = traced("save_errors_arrays", inout.save_errors_arrays)

  def timeline(t0):
    agg = {}
    for name, a0, a1 in tl:
      g = agg.setdefault(name, [a0, a1, 0.0, 0])
      g[0], g[1] = min(g[0], a0), max(g[1], a1)
      g[2] += a1 - a0
      g[3] += 1
    return {k: {"first_start": round(v[0] - t0, 3), "last_end": round(v[1] - t0, 3),
                "busy": round(v[2], 3), "n": v[3]} for k, v in sorted(agg.items(),
                                                                    key=lambda kv: kv[1][0])}
  for mod, name in ((ece, "scene_records"), (ece, "scene_arrays_direct"), (ece, "plan_rank"),
                    (ece, "load_scene_depths"),
                    (ece, "evaluate_batch"), (ece, "evaluate"), (ece, "Models"), (inout, "save_json"), (inout, "save_json_per_value")):
    setattr(mod, name, timed("host:" + name, getattr(mod, name)))
  p = eval_bop19_pose.parse_args([
      "--result_filenames", result, "--results_path", os.path.join(a.root, "results"),
      "--eval_path", os.path.join(a.root, "eval")])
  prof = None
  if a.profile:
    import cProfile
    prof = cProfile.Profile()
    prof.enable()
  t0 = time.perf_counter()
  marks.clear()
  tl.clear()
  final = eval_bop19_pose.evaluate(p)
  t_eval = time.perf_counter() - t0
  first_tail = tail_info(t0 + t_eval)
  first_timeline = timeline(t0)
  first_events = [(nm, round(e0 - t0, 4), round(e1 - t0, 4))
                  for nm, e0, e1 in sorted(tl, key=lambda x: x[1])]
  if prof is not None:
    import io
    import pstats
    prof.disable()
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("cumulative").print_stats(45)
    pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(30)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "e2e_profile.txt"), "w") as f:
      f.write(s.getvalue())
  scores = final[os.path.splitext(result)[0]]
  first_stats = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in depth_gpu.STATS.items()}
  ab = None
  if a.ab_depth:  # warm runs (annotation caches filled by the first): host decoder, then GPU
    first_phases, first_err = dict(phases), dict(err_t)
    ab = {}
    runs = (("host_decode_warm", "0", None), ("gpu_decode_warm", "1", None))
    if a.ab_group:  # decode launches per scene (0) vs shared launches of ~G frames
      gs = a.ab_group.split(",")
      runs = tuple(("gpu_decode_group%s_warm%d" % (g, r), "1", g)
                   for r in range(1, a.warm_reps + 1) for g in gs)
    for name, env, grp in runs:
      if grp is None:
        os.environ.pop("BOPX_DEPTH_GROUP_FRAMES", None)
      else:
        os.environ["BOPX_DEPTH_GROUP_FRAMES"] = grp
      for k in list(phases):
        if k.startswith("host:"):
          phases[k] = 0.0
      err_t.clear()
      for k in depth_gpu.STATS:
        depth_gpu.STATS[k] = 0 if k in ("calls", "frames") else 0.0
      os.environ["BOPX_DEPTH_GPU"] = env
      t0 = time.perf_counter()
      marks.clear()
      tl.clear()
      fin = eval_bop19_pose.evaluate(p)
      t_run = time.perf_counter() - t0
      ab[name] = {"eval_bop19_s": round(t_run, 2), "tail": tail_info(t0 + t_run),
                  "depth_decoder": {k: (round(v, 3) if isinstance(v, float) else v)
                                    for k, v in depth_gpu.STATS.items()},
                  "errors_s": {k: round(v, 2) for k, v in err_t.items()},
                  "host_s": {k[5:]: round(v, 3) for k, v in phases.items()
                             if k.startswith("host:") and v},
                  "eval_tuples_per_s": n / t_run,
                  "identical_scores": fin[os.path.splitext(result)[0]] == scores,
                  "timeline": timeline(t0),
                  # the host steps one by one (name, start, end; s from the run's start)
                  "events": [(nm, round(e0 - t0, 4), round(e1 - t0, 4))
                             for nm, e0, e1 in sorted(tl, key=lambda x: x[1])]}
    os.environ.pop("BOPX_DEPTH_GPU")
    os.environ.pop("BOPX_DEPTH_GROUP_FRAMES", None)
    phases.clear()
    phases.update(first_phases)
    err_t.clear()
    err_t.update(first_err)
  print(json.dumps({
      "what": "end-to-end BOP19 evaluation (calc_gt_info + eval_bop19_pose), synthetic YCB-V "
              "layout, 21 objs V=5002, 640x480 PNG depth, 1 GPU",
      "images": a.images, "instances": a.instances, "tuples": n, "gen_s": round(t_gen, 2),
      "shared_render_ratio": ece.SHARED_RENDER_RATIO,
      "calc_gt_info_s": round(phases["calc_gt_info"], 2),
      "errors_s": {k: round(v, 2) for k, v in err_t.items()},
      "scores_s": round(phases.get("scores", 0.0), 2), "eval_bop19_s": round(t_eval, 2),
      "host_s": {k[5:]: round(v, 3) for k, v in phases.items() if k.startswith("host:")},
      "eval_tuples_per_s": n / t_eval,
      "depth_decoder": "gpu" if depth_gpu.enabled() else "host", "ab_depth": ab,
      "depth_decoder_first_run": first_stats, "depth_decoder_gt_info": gt_stats, "tail": first_tail, "timeline": first_timeline,
      "events": first_events,
      "ar": {k: round(float(v), 4) for k, v in scores.items()}}))


if __name__ == "__main__":
  main()
