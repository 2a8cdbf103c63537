#!/usr/bin/env python
"""BOP19 pose-error throughput on MI355X: VSD (10 taus) + MSSD + MSPD tuples/s.

One step = the full BOP19 error set of every (est, gt) tuple of a synthetic
job (BASELINE.json configs[3]): 21 LM-O/YCB-V-like objects (5,002 verts /
10,000 faces, S in {1,2,4,8} + one continuous-symmetry object with S = 314),
640x480 test depth, YCB-V intrinsics, 6 objects per image, 100,002 tuples
(16,667 images) in total. Inputs are resident in HBM before timing; each step
runs k_vsd (both renders + VSD fused), k_sym_error<MSSD> and
k_sym_error<MSPD>, and for N > 1 one RCCL gather of the per-tuple error rows
to rank 0. Strong scaling: the configuration's tuple count is fixed and its
images are split over the ranks by LPT on the SURVEY.md §8d cost model
(shard.lpt_shard; tuples are independent).

    python bench.py [--gpus N --steps K --warmup W --config C --tuples T]
    torchrun --nproc-per-node N bench.py --gpus N ...

`python bench.py --gpus N` (no torchrun) starts the N rank processes itself
(launch_ranks: one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as
torchrun sets them) and exits with their status; under torchrun WORLD_SIZE
must equal N.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

N_TAU = 10
TAUS = np.arange(0.05, 0.51, 0.05)
DELTA = 15.0
W, H = 640, 480
# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level table)
HBM_PEAK_GBS = 8000.0
FP64_PEAK_TF = 78.6
FP32_PEAK_TF = 157.3


# BASELINE.json configs (index): the whole job each names (tuples in total,
# split over the ranks). Default: configs[3], the metric's configuration
# (BOP19 set, 100k est).
CONFIGS = {
    0: {"objects": 1, "n_lat": 25, "n_lon": 40, "syms": [1], "continuous": False,
        "tuples": 100, "K": "LMO_K", "W": 640, "H": 480, "errors": ("add", "adi"),
        "what": "configs[0]: ADD/ADI, 1 LM-O-like obj ~1k verts, 100 est/gt pairs"},
    1: {"objects": 8, "n_lat": 50, "n_lon": 100, "syms": [1, 2, 4, 8], "continuous": False,
        "tuples": 10000, "K": "LMO_K", "W": 640, "H": 480, "errors": ("mssd", "mspd"),
        "what": "configs[1]: MSSD+MSPD, 8 LM-O-like objs, S<=8, 10k est"},
    2: {"objects": 21, "n_lat": 50, "n_lon": 100, "syms": [1, 2, 4, 8], "continuous": True,
        "tuples": 50000, "K": "YCBV_K", "W": 640, "H": 480, "errors": ("vsd",),
        "what": "configs[2]: VSD (10 taus) with HIP raster, 21 YCB-V-like objs, 50k est"},
    3: {"objects": 21, "n_lat": 50, "n_lon": 100, "syms": [1, 2, 4, 8], "continuous": True,
        "tuples": 100000, "K": "YCBV_K", "W": 640, "H": 480, "errors": ("vsd", "mssd", "mspd"),
        "what": "BASELINE configs[3]: BOP19 error set (VSD 10 taus + MSSD + MSPD), 100k est"},
    4: {"objects": 30, "n_lat": 100, "n_lon": 150, "syms": [1, 2, 4, 8, 16, 32, 64],
        "continuous": False, "tuples": 200000, "K": "TLESS_K", "W": 720, "H": 540,
        "errors": ("vsd", "mssd", "mspd"),
        "what": "configs[4]: T-LESS-like BOP19 set, ~15k verts, S<=64, 200k est"},
    # Multi-instance variant of configs[4] (T-LESS / IC-BIN / ITODD images hold
    # several instances of an object; n_top = -1 pairs every estimate with every
    # GT instance, eval_calc_errors.py:281-290): 3 objects per image with k in
    # [3, 6] instances and k estimates each, k^2 tuples per (image, object). VSD
    # runs on shared renders (each distinct pose rasterised once, k_vsd_pair per
    # tuple); the fused per-tuple k_vsd on the same tuples is timed beside it.
    5: {"objects": 30, "n_lat": 100, "n_lon": 150, "syms": [1, 2, 4, 8, 16, 32, 64],
        "continuous": False, "tuples": 100000, "K": "TLESS_K", "W": 720, "H": 540,
        "errors": ("vsd", "mssd", "mspd"), "multi": (3, 3, 6),
        "what": "configs[4] multi-instance variant: 3 objs/image x k in [3,6] instances, "
                "k^2 tuples each (n_top -1), shared renders"},
}


def parse():
  ap = argparse.ArgumentParser()
  ap.add_argument("--gpus", type=int, default=1)
  ap.add_argument("--steps", type=int, default=10)
  ap.add_argument("--warmup", type=int, default=2)
  ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS),
                  help="BASELINE.json configs index (3 = the metric's workload)")
  ap.add_argument("--tuples", type=int, default=None,
                  help="tuples of the whole job (split over the ranks)")
  ap.add_argument("--objects", type=int, default=None)
  ap.add_argument("--n-lat", type=int, default=None)
  ap.add_argument("--n-lon", type=int, default=None)
  ap.add_argument("--axes-scale", type=float, default=1.0,
                  help="object size factor (design experiments; 1 = the configuration's)")
  ap.add_argument("--cpu-seconds", type=float, default=10.0,
                  help="target wall time of the CPU-baseline sample")
  ap.add_argument("--no-cpu-baseline", action="store_true",
                  help="skip the oracle legs after the timed region (cpu_baseline and parity)")
  ap.add_argument("--no-parity", action="store_true",
                  help="skip the post-timed-region parity leg (every config vs the oracle)")
  ap.add_argument("--e2e-images", type=int, default=None,
                  help="images of the end-to-end drop-in run after the timed region (default "
                       "16,667 = the whole configs[3] job at N=1, else 0 = none)")
  ap.add_argument("--seed", type=int, default=20250220 + 4)
  args = ap.parse_args()
  cfg = CONFIGS[args.config]
  for k in ("tuples", "objects", "n_lat", "n_lon"):
    if getattr(args, k) is None:
      setattr(args, k, cfg[k])
  global W, H
  W, H = cfg["W"], cfg["H"]
  args.cfg = cfg
  return args


def build_objects(ev, args, torch, dia_device=None):
  from bop_toolkit_amd import misc, synth
  rng = np.random.default_rng(args.seed)
  objs = []
  for o in range(args.objects):
    axes = tuple(args.axes_scale * rng.uniform(30.0, 100.0, 3))
    pts, faces = synth.superellipsoid(args.n_lat, args.n_lon, axes, float(rng.uniform(0.5, 1.0)))
    # exact diameter (max pairwise distance) on the host, in row chunks: set-up
    # only, kept off the GPU so the profile holds the measured kernels alone
    # (the parity leg, after the timed region, takes it on dia_device)
    p = torch.as_tensor(pts, device=dia_device)
    dia = max(float(torch.cdist(p[i:i + 2048], p, compute_mode="donot_use_mm_for_euclid_dist").max())
              for i in range(0, len(p), 2048))
    info = {"diameter": dia}
    if o == args.objects - 1 and args.cfg["continuous"]:
      info["symmetries_continuous"] = [{"axis": [0, 0, 1], "offset": [0, 0, 0]}]
    else:
      pat = args.cfg["syms"]
      n_disc = pat[o % len(pat)]
      info["symmetries_discrete"] = [
          np.concatenate([np.concatenate([synth.rot_z(2 * np.pi * j / n_disc), np.zeros((3, 1))],
                                         1), [[0, 0, 0, 1]]]).reshape(-1).tolist()
          for j in range(1, n_disc)]
    syms = misc.get_symmetry_transformations(info, 0.01)
    ev.add_object(o, pts, faces, syms, dia)
    objs.append({"pts": pts, "faces": faces, "syms": misc.symmetries_to_array(syms),
                 "diameter": dia, "bbox": (pts.min(0), pts.max(0))})
  return objs


def build_workload(ev, objs, args, rank, world, torch):
  """The whole job's images (6 objects each), identical for every N, and this
  rank's LPT shard of them. Test depth = composite GT render + background
  plane + occluder + noise + 10 % holes, rounded to integer mm (uint16 PNG),
  synthesised on the GPU in chunks of images (bounded temporaries)."""
  from bop_toolkit_amd import shard, synth
  rng = np.random.default_rng(args.seed + 1000)
  per_img = min(6, len(objs))
  n_img_all = (args.tuples + per_img - 1) // per_img
  n_all = n_img_all * per_img
  obj_all = np.stack([rng.choice(len(objs), per_img, replace=False)
                      for _ in range(n_img_all)]).reshape(-1).astype(np.int32)
  Rg, tg = synth.gt_poses(rng, n_all)
  Re, te = synth.perturb(rng, Rg, tg)
  pe_all = np.concatenate([Re.reshape(n_all, 9), te], 1)
  pg_all = np.concatenate([Rg.reshape(n_all, 9), tg], 1)
  K = getattr(synth, args.cfg["K"])
  if world > 1:
    # LPT over images on the SURVEY §8d per-tuple cost (shard.tuple_cost)
    roi = roi_pixels(objs, obj_all, [pe_all, pg_all], K)
    nv = np.array([len(objs[o]["pts"]) for o in obj_all])
    nf = np.array([len(objs[o]["faces"]) for o in obj_all])
    ns = np.array([len(objs[o]["syms"]) for o in obj_all])
    cost = shard.image_costs(np.repeat(np.arange(n_img_all), per_img),
                             shard.tuple_cost(nv, nf, ns, roi), n_img_all)
    parts = shard.lpt_shard(cost, world)
  else:
    parts = [np.arange(n_img_all)]
  mine = parts[rank]
  counts = [len(p) * per_img for p in parts]
  gid = (mine[:, None] * per_img + np.arange(per_img)).reshape(-1)
  n_img, n = len(mine), len(gid)
  obj, pe, pg = obj_all[gid], pe_all[gid], pg_all[gid]
  frame_idx = np.repeat(np.arange(n_img, dtype=np.int32), per_img)
  cam = np.tile([K[0, 0], K[1, 1], K[0, 2], K[1, 2]], (n_img, 1)).astype(np.float64)
  dev = ev.device
  t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
  d = {"slots": ev.slots(obj), "pose_est": t(pe, torch.float64), "pose_gt": t(pg, torch.float64),
       "frame_idx": t(frame_idx, torch.int32), "cam": t(cam, torch.float64),
       "K": t(np.tile(K.reshape(9), (n, 1)), torch.float64),
       "diameters": t([objs[o]["diameter"] for o in obj], torch.float64),
       "gid": t(gid, torch.int64), "counts": counts, "n_total": n_all}
  frames = ev.render(d["slots"], d["pose_gt"], d["frame_idx"], d["cam"], n_img, W, H)
  g = torch.Generator(device=dev)
  g.manual_seed(args.seed + rank)
  ys = torch.arange(H, device=dev).view(1, H, 1)
  xs = torch.arange(W, device=dev).view(1, 1, W)
  for c0 in range(0, n_img, 2048):
    f = frames[c0:c0 + 2048]
    m = f.shape[0]
    f[f <= 0] = 1600.0  # background plane
    # one occluder rectangle per image in front of the scene
    x0 = torch.randint(0, W - 120, (m, 1, 1), device=dev, generator=g)
    y0 = torch.randint(0, H - 120, (m, 1, 1), device=dev, generator=g)
    sz = torch.randint(40, 120, (m, 1, 1), device=dev, generator=g)
    occ = (xs >= x0) & (xs < x0 + sz) & (ys >= y0) & (ys < y0 + sz)
    f.masked_fill_(occ, 450.0)
    f.add_(torch.randn(f.shape, device=dev, generator=g), alpha=2.0)
    f.round_().clamp_(0, 65535)
    f.masked_fill_(torch.rand(f.shape, device=dev, generator=g) < 0.1, 0.0)
  d["frames"] = frames
  d["host"] = {"obj": obj, "pe": pe, "pg": pg, "frame_idx": frame_idx, "cam": cam}
  torch.cuda.synchronize()
  return n, d


def plan_multi(cfg, meta, tuples, seed, rank, world, K, width, height):
  """Host plan of the multi-instance workload (configs[5]): images with m
  objects, k instances of each (k uniform in [kmin, kmax]) and k estimates
  per (image, object); tuples = every estimate x every GT instance of its
  object (k^2 per (image, object), eval_calc_errors.py:281-290). The whole
  job is generated identically on every rank; images are then assigned to
  the ranks by LPT on the SURVEY.md §8d per-tuple cost (shard.tuple_cost) —
  the k^2 tuples per image vary 9x, so contiguous ranges would not balance.
  meta: per object {"nv", "nf", "ns", "bbox": (lo, hi)}. Returns this rank's
  tuples (global ids, local frame index), its GT instances, and every rank's
  tuple count."""
  from bop_toolkit_amd import shard, synth
  m, kmin, kmax = cfg["multi"]
  rng = np.random.default_rng(seed + 2000)
  per_img_mean = m * np.mean([k * k for k in range(kmin, kmax + 1)])
  n_img_all = int(np.ceil(tuples / per_img_mean))
  i_img, i_obj, i_pose = [], [], []  # GT instances
  t_img, t_obj, t_pe, t_pg = [], [], [], []  # tuples, global id = position
  for f in range(n_img_all):
    for o in rng.choice(len(meta), m, replace=False):
      k = int(rng.integers(kmin, kmax + 1))
      Rg, tg = synth.gt_poses(rng, k)
      Re, te = synth.perturb(rng, Rg, tg)
      pg = np.concatenate([Rg.reshape(k, 9), tg], 1)
      pe = np.concatenate([Re.reshape(k, 9), te], 1)
      i_img += [f] * k
      i_obj += [int(o)] * k
      i_pose.append(pg)
      t_img += [f] * (k * k)
      t_obj += [int(o)] * (k * k)
      t_pe.append(np.repeat(pe, k, axis=0))  # estimate i x GT j, i major
      t_pg.append(np.tile(pg, (k, 1)))
  t_img, t_obj = np.array(t_img, np.int64), np.array(t_obj, np.int32)
  t_pe, t_pg = np.concatenate(t_pe), np.concatenate(t_pg)
  i_img, i_obj, i_pose = np.array(i_img, np.int64), np.array(i_obj, np.int32), np.concatenate(i_pose)
  n_all = len(t_img)
  if world > 1:
    lo = np.stack([meta[o]["bbox"][0] for o in t_obj])
    hi = np.stack([meta[o]["bbox"][1] for o in t_obj])
    roi = shard.roi_pixels(lo, hi, [t_pe, t_pg], K, width, height)
    nv, nf, ns = (np.array([meta[o][k] for o in t_obj]) for k in ("nv", "nf", "ns"))
    parts = shard.lpt_shard(shard.image_costs(t_img, shard.tuple_cost(nv, nf, ns, roi),
                                              n_img_all), world)
  else:
    parts = [np.arange(n_img_all)]
  per_img = np.bincount(t_img, minlength=n_img_all)
  mine = parts[rank]
  sel = np.nonzero(np.isin(t_img, mine))[0]
  isel = np.nonzero(np.isin(i_img, mine))[0]
  return {"gid": sel, "obj": t_obj[sel], "frame_idx": np.searchsorted(mine, t_img[sel]).astype(
              np.int32), "pe": t_pe[sel], "pg": t_pg[sel],
          "inst_obj": i_obj[isel], "inst_f": np.searchsorted(mine, i_img[isel]).astype(np.int32),
          "inst_pose": i_pose[isel], "n_img": len(mine), "n_all": n_all,
          "counts": [int(per_img[p].sum()) for p in parts]}


def build_workload_multi(ev, objs, args, rank, world, torch):
  """configs[5] on this rank (plan_multi: LPT shard of the images). Test depth
  as in build_workload, composited from every GT instance."""
  from bop_toolkit_amd import synth
  from bop_toolkit_amd.batch import unique_renders
  K = getattr(synth, args.cfg["K"])
  meta = [{"nv": len(o["pts"]), "nf": len(o["faces"]), "ns": len(o["syms"]), "bbox": o["bbox"]}
          for o in objs]
  pl = plan_multi(args.cfg, meta, args.tuples, args.seed, rank, world, K, W, H)
  obj, frame_idx, pe, pg, n_img = pl["obj"], pl["frame_idx"], pl["pe"], pl["pg"], pl["n_img"]
  n = len(obj)
  cam = np.tile([K[0, 0], K[1, 1], K[0, 2], K[1, 2]], (n_img, 1)).astype(np.float64)
  dev = ev.device
  t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
  ro, rp, rf, er, gr = unique_renders(obj, pe, pg, frame_idx)
  d = {"slots": ev.slots(obj), "pose_est": t(pe, torch.float64), "pose_gt": t(pg, torch.float64),
       "frame_idx": t(frame_idx, torch.int32), "cam": t(cam, torch.float64),
       "K": t(np.tile(K.reshape(9), (n, 1)), torch.float64),
       "diameters": t([objs[o]["diameter"] for o in obj], torch.float64),
       "gid": t(pl["gid"], torch.int64), "n_total": pl["n_all"], "counts": pl["counts"],
       "renders": {"slots": ev.slots(ro), "pose": t(rp, torch.float64),
                   "frame_idx": t(rf, torch.int32), "est": t(er, torch.int32),
                   "gt": t(gr, torch.int32), "n": len(ro)}}
  frames = ev.render(ev.slots(pl["inst_obj"]), t(pl["inst_pose"], torch.float64),
                     t(pl["inst_f"], torch.int32), d["cam"], n_img, W, H)
  g = torch.Generator(device=dev)
  g.manual_seed(args.seed + rank)
  for c0 in range(0, n_img, 1024):
    f = frames[c0:c0 + 1024]
    f[f <= 0] = 1600.0
    f.add_(torch.randn(f.shape, device=dev, generator=g), alpha=2.0)
    f.round_().clamp_(0, 65535)
    f.masked_fill_(torch.rand(f.shape, device=dev, generator=g) < 0.1, 0.0)
  d["frames"] = frames
  d["host"] = {"obj": obj, "pe": pe, "pg": pg, "frame_idx": frame_idx, "cam": cam}
  torch.cuda.synchronize()
  return n, d


def roi_pixels(objs, obj, poses, K):
  """Survey §8d ROI per tuple (shard.roi_pixels)."""
  from bop_toolkit_amd import shard
  lo = np.stack([objs[o]["bbox"][0] for o in obj])
  hi = np.stack([objs[o]["bbox"][1] for o in obj])
  return shard.roi_pixels(lo, hi, poses, K, W, H)


def algorithmic_cost(objs, host, n, K):
  """Compulsory HBM bytes and VALU flops per launch (SURVEY.md §8d formulas)."""
  obj = host["obj"]
  roi = roi_pixels(objs, obj, [host["pe"], host["pg"]], K)
  used = np.unique(obj)
  V = np.array([len(objs[o]["pts"]) for o in obj], np.float64)
  F = np.array([len(objs[o]["faces"]) for o in obj], np.float64)
  S = np.array([len(objs[o]["syms"]) for o in obj], np.float64)
  mesh_bytes = sum(12 * len(objs[o]["pts"]) + 12 * len(objs[o]["faces"]) for o in used)
  sym_bytes = sum(96 * len(objs[o]["syms"]) for o in used)
  vsd_bytes = n * (192 + 16 + 8 * N_TAU) + 4.0 * roi.sum() + mesh_bytes
  vsd_f32 = (40 * V + 60 * F + 34 * roi).sum()
  vsd_f64 = (58 * roi).sum()
  mssd_bytes = n * (192 + 4 + 8) + sum(24 * len(objs[o]["pts"]) for o in used) + sym_bytes
  mspd_bytes = mssd_bytes + n * 72
  mssd_f64 = (V * (18 + 28 * S)).sum()
  mspd_f64 = (V * (20 + 27 * S)).sum()
  pts_bytes = n * (192 + 4 + 8) + sum(24 * len(objs[o]["pts"]) for o in used)
  add_f64 = (46 * V).sum()
  adi_f64 = (36 * V + 9 * V * V).sum()  # brute-force NN
  return {"add": (pts_bytes, 0.0, add_f64), "adi": (pts_bytes, 0.0, adi_f64),
          "vsd": (vsd_bytes, vsd_f32, vsd_f64), "mssd": (mssd_bytes, 0.0, mssd_f64),
          "mspd": (mspd_bytes, 0.0, mspd_f64), "roi_mean": float(roi.mean())}


def free_port():
  import socket
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  port = s.getsockname()[1]
  s.close()
  return port


def rank_envs(n, port, base=None):
  """The environment of each of n rank processes on this node (what
  torch.distributed.run exports), rendezvous on 127.0.0.1."""
  base = dict(os.environ if base is None else base)
  return [dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
          for r in range(n)]


def launch_ranks(cmd, n, base_env=None, poll=0.2):
  """Run cmd as n rank processes (rank_envs) and wait for them. If one fails,
  the others are terminated (their own pids, then killed after 30 s). Returns
  0 or the first failing rank's exit status. The caller must not have touched
  the GPU (the children initialise it)."""
  import subprocess
  envs = rank_envs(n, free_port(), base_env)
  procs = [subprocess.Popen(cmd, env=e) for e in envs]
  rc = 0
  try:
    live = list(procs)
    while live:
      time.sleep(poll)
      for p in list(live):
        r = p.poll()
        if r is None:
          continue
        live.remove(p)
        if r != 0 and rc == 0:
          rc = r if r > 0 else 128 - r
          print("bench.py: rank %d exited with status %d; stopping the other %d rank(s)" %
                (procs.index(p), r, len(live)), file=sys.stderr, flush=True)
          for q in live:
            q.terminate()
  finally:
    for p in procs:
      try:
        p.wait(timeout=30)
      except subprocess.TimeoutExpired:
        p.kill()
        p.wait()
  return rc


def world_of(args, environ=None):
  """(rank, world, local_rank) of this process; None when this is the
  launcher of --gpus N > 1 rank processes (no WORLD_SIZE in the
  environment). Under torchrun WORLD_SIZE must equal --gpus."""
  env = os.environ if environ is None else environ
  if "WORLD_SIZE" not in env:
    if args.gpus > 1:
      return None
    return 0, 1, 0
  world = int(env["WORLD_SIZE"])
  if world != args.gpus:
    raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
  return int(env.get("RANK", 0)), world, int(env.get("LOCAL_RANK", 0))


def lib_digest():
  """sha256 of the loaded libbopx.so: ties a PMC summary to the build it measured."""
  import hashlib
  from bop_toolkit_amd import _lib
  with open(_lib.LIB_PATH, "rb") as f:
    return hashlib.sha256(f.read()).hexdigest()


def code_digests():
  """sha256 of the gfx950 code objects holding the measured kernels
  (_lib.code_object_digests): ties a PMC summary to the machine code it
  counted, not to the whole library (host code and other kernels' code
  objects may change without changing these)."""
  from bop_toolkit_amd import _lib
  d = _lib.code_object_digests()
  return {k: d.get(k) for k in ("k_vsd", "k_sym_error", "k_mean_error", "k_adi")}


def workload_key(args, n):
  return "config=%d tuples=%d objects=%d n_lat=%d n_lon=%d axes_scale=%g seed=%d" % (
      args.config, n, args.objects, args.n_lat, args.n_lon, args.axes_scale, args.seed)


def load_traffic(dom, args, n):
  """HBM bytes per launch of kernel `dom` from the committed rocprofv3 PMC
  summaries (profiles/*_pmc.json, written by tools/pmc_summary.py), or None.
  A summary counts only if it records the code object of the measured kernel
  (`code_sha256`, or a whole-library `lib_sha256` equal to this one) and this
  launch's workload (`workload`): otherwise it measured something else."""
  import glob
  name = {"vsd": "k_vsd", "mssd": "k_sym_error<MSSD>", "mspd": "k_sym_error<MSPD>"}.get(dom)
  if name is None:
    return None
  family = name.split("<")[0]
  code = code_digests().get(family)
  digest, key = lib_digest(), workload_key(args, n)
  best = None
  for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc.json"))):
    try:
      with open(path) as f:
        j = json.load(f)
    except (OSError, ValueError):
      continue
    meta = j.get("_meta", {})
    same_code = code is not None and meta.get("code_sha256", {}).get(family) == code
    if (same_code or meta.get("lib_sha256") == digest) and meta.get("workload") == key:
      best = j.get(name, {}).get("hbm_bytes_per_launch", best)
  return best


def cpu_baseline(objs, d, n, seconds, gpu=None):
  """Oracle (C restatement of the reference per-tuple algorithm: two full-frame
  renders, three full-frame distance images, per-symmetry loops) on the host
  cores, OpenMP over tuples, on a bounded sample of the same workload. gpu:
  the timed steps' (vsd, mssd, mspd) outputs, checked against the oracle's
  results for the sample (`check`: VSD rows bit-identical, largest MSSD / MSPD
  relative difference)."""
  threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)), 16))
  os.environ["OMP_NUM_THREADS"] = str(threads)
  from oracle import oracle
  h = d["host"]
  frames = d["frames"]

  def run(m):
    fidx = h["frame_idx"][:m]
    used = np.unique(fidx)
    remap = np.searchsorted(used, fidx).astype(np.int32)
    fr = frames[used.tolist()].cpu().numpy()
    t0 = time.perf_counter()
    res = oracle.bop19_batch(objs, h["obj"][:m], h["pe"][:m], h["pg"][:m], remap, fr,
                             h["cam"][used], DELTA, TAUS,
                             np.array([objs[o]["diameter"] for o in h["obj"][:m]]))
    return time.perf_counter() - t0, res

  m0 = min(n, 2 * threads)
  t0, _ = run(m0)
  m = int(min(n, max(m0, m0 * seconds / max(t0, 1e-3))))
  t1, (ov, om, op) = run(m)
  if t1 < 0.8 * seconds and m < n:  # the small first sample over-estimated the per-tuple time
    m = int(min(n, m * seconds / max(t1, 1e-3)))
    t1, (ov, om, op) = run(m)
  out = {"value": m / t1, "unit": "tuples/s", "cores": threads, "kind": "port",
         "sample": "%d tuples (first %d of this rank's workload), BOP19 set, %.1f s wall; "
                   "oracle/bopx_oracle.c, reference per-tuple algorithm in C" % (m, m, t1),
         # the reference itself cannot travel to the GPU box; its own NumPy path was
         # timed in the survey container
         "reference_survey": {"value": 79.0, "unit": "tuples/s/core",
                              "note": "reference NumPy path (pose_error.py), full BOP19 tuple "
                                      "V=5k S=8 excluding the raster (no OpenGL offline), 1 "
                                      "Xeon core of the survey container, BASELINE.md §2"}}
  if gpu is not None:
    gv, gm, gp = (t[:m].cpu().numpy() for t in gpu)

    def rel(a, b):
      fin = np.isfinite(a) & np.isfinite(b)
      same_inf = np.array_equal(np.isfinite(a), np.isfinite(b)) and np.array_equal(a[~fin],
                                                                                  b[~fin])
      r = np.abs(a[fin] - b[fin]) / np.maximum(np.abs(b[fin]), 1e-300)
      return float(r.max()) if r.size and same_inf else (0.0 if same_inf else float("inf"))
    out["check"] = {"tuples": m, "vsd_rows_bit_identical": int((gv == ov).all(1).sum()),
                    "mssd_max_rel": rel(gm, om), "mspd_max_rel": rel(gp, op),
                    "note": "this run's GPU outputs vs the oracle on the sample (the checker)"}
  return out


def e2e_run(images, seed, timeout=300):
  """The drop-in evaluation end to end, after the timed region: a YCB-V-layout
  dataset of `images` 640x480 images with 6 of configs[3]'s kind of objects
  each (21 superellipsoids of 5,002 vertices, Pillow-written 16-bit depth
  PNGs, a BOP19 results CSV) written to local disk, then calc_gt_info and ONE
  cold eval_bop19_pose (VSD + MSSD + MSPD errors and the 120 score settings)
  in a fresh process (tools/e2e_bench.py, a child of this one). Returns the
  child's JSON summary (tuples/s of eval_bop19_pose, phases, recalls)."""
  import shutil
  import subprocess
  root = os.path.join(os.environ.get("TMPDIR", "/tmp"), "bopx_bench_e2e_%d" % os.getpid())
  try:
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "e2e_bench.py"), "--images",
                        str(images), "--root", root, "--seed", str(seed)],
                       capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
      return {"error": "e2e_bench exit %d: %s" % (r.returncode, r.stderr[-400:])}
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
  except (subprocess.TimeoutExpired, ValueError, IndexError) as e:
    return {"error": repr(e)[:400]}
  finally:
    shutil.rmtree(root, ignore_errors=True)
  keep = ("images", "tuples", "eval_bop19_s", "eval_tuples_per_s", "calc_gt_info_s", "errors_s",
          "tail", "host_s", "gen_s", "depth_decoder", "depth_decoder_first_run", "ar")
  res = {k: out[k] for k in keep if k in out}
  res["note"] = ("cold: one drop-in eval_bop19_pose (errors VSD/MSSD/MSPD + 120 score settings) "
                 "in a fresh process on PNG files on local disk; tuples/s = its tuples / its wall "
                 "time; calc_gt_info separate")
  return res


# tuples per configuration in the parity leg (a few hundred of each workload)
PARITY_TUPLES = {0: 100, 1: 600, 2: 300, 3: 300, 4: 240, 5: 300}
PARITY_TOL = 1e-4  # north_star: within 1e-4 mm / 1e-4 px of the reference


def _max_diff(a, b):
  """(max abs, max rel) difference of two float64 vectors whose infinities
  must coincide (gated / empty-set values); inf when they do not."""
  a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
  fa, fb = np.isfinite(a), np.isfinite(b)
  if not (np.array_equal(fa, fb) and np.array_equal(a[~fa], b[~fb])):
    return float("inf"), float("inf")
  if not fa.any():
    return 0.0, 0.0
  d = np.abs(a[fa] - b[fa])
  return float(d.max()), float((d / np.maximum(np.abs(b[fa]), 1e-300)).max())


def parity_leg(args, torch, skip=(), png_frames=None):
  """After the timed region (rank 0, N = 1): a few hundred tuples of every
  BASELINE.json configuration's own workload generator (build_objects /
  build_workload / build_workload_multi with that configuration's objects,
  camera and image size) through the HIP path, checked against the CPU oracle
  (oracle/bopx_oracle.c, the checker): VSD rows bit-identical, MSSD / MSPD /
  ADD / ADI within PARITY_TOL with matching infinities; then test-depth PNGs
  (Pillow-written, several zlib levels) decoded by kern_png.hip vs Pillow, bit
  for bit, with no frame left to the host decoder. `skip`: configurations
  already checked by this run (cpu_baseline.check)."""
  global W, H
  from bop_toolkit_amd import synth
  from bop_toolkit_amd.batch import BatchEvaluator
  from oracle import oracle
  t_all = time.perf_counter()
  keep_wh = (W, H)
  res, ok = {}, True
  png_src = [png_frames]
  try:
    for c in sorted(PARITY_TUPLES):
      if c in skip:
        continue
      try:
        ok &= parity_config(c, args, torch, oracle, synth, BatchEvaluator, res, png_src)
      except Exception as e:  # noqa: BLE001 - reported in the line, the bench line still prints
        res[str(c)] = {"error": repr(e)[:300]}
        ok = False
      torch.cuda.empty_cache()
  finally:
    W, H = keep_wh
  png_frames = png_src[0]
  png = None
  if png_frames is not None:
    try:
      png = png_check(png_frames, torch)
      ok &= png["bit_identical"] == png["frames"] and png["device_decoded"] == png["frames"]
    except Exception as e:  # noqa: BLE001
      png = {"error": repr(e)[:300]}
      ok = False
  torch.cuda.empty_cache()
  return {"configs": res, "png": png, "all_ok": bool(ok), "tol": PARITY_TOL,
          "s": round(time.perf_counter() - t_all, 2),
          "note": "HIP path vs the CPU oracle (oracle/bopx_oracle.c, the checker) on each "
                  "BASELINE.json configuration's own generator (configs index as key; 5 = the "
                  "multi-instance shared-render variant); VSD rows compared bit for bit, point "
                  "errors by max abs / rel with matching infinities; png: kern_png.hip vs "
                  "Pillow on 16-bit PNGs of configs[3] test depth"}


def parity_config(c, args, torch, oracle, synth, BatchEvaluator, res, png_src):
  """One configuration of the parity leg (parity_leg); records its row in res
  and returns whether it passed (png_src: [frames or None], filled from
  configs[3] when the caller has no test depth for the PNG check)."""
  global W, H
  import copy
  t0 = time.perf_counter()
  ok = True
  cfg = CONFIGS[c]
  a = copy.copy(args)
  a.config, a.cfg, a.tuples, a.axes_scale = c, cfg, PARITY_TUPLES[c], 1.0
  a.objects, a.n_lat, a.n_lon = cfg["objects"], cfg["n_lat"], cfg["n_lon"]
  a.seed = 20250220 + 4
  W, H = cfg["W"], cfg["H"]
  ev = BatchEvaluator(0)
  objs = build_objects(ev, a, torch, dia_device=ev.device)
  multi = "multi" in cfg
  n, d = (build_workload_multi if multi else build_workload)(ev, objs, a, 0, 1, torch)
  h = d["host"]
  errs = cfg["errors"]
  got = {}
  if "vsd" in errs:
    rd = d.get("renders")
    got["vsd"] = (ev.vsd_shared(rd["slots"], rd["pose"], rd["frame_idx"], rd["est"], rd["gt"],
                                d["frames"], d["cam"], DELTA, TAUS, d["diameters"]) if multi
                  else ev.vsd(d["slots"], d["pose_est"], d["pose_gt"], d["frame_idx"],
                              d["frames"], d["cam"], DELTA, TAUS, d["diameters"]))
  if "mssd" in errs:
    got["mssd"] = ev.mssd(d["slots"], d["pose_est"], d["pose_gt"])
    got["mspd"] = ev.mspd(d["slots"], d["pose_est"], d["pose_gt"], d["K"])
  if "add" in errs:
    got["add"] = ev.add(d["slots"], d["pose_est"], d["pose_gt"])
    got["adi"] = ev.adi(d["slots"], d["pose_est"], d["pose_gt"])
  torch.cuda.synchronize()
  got = {k: v.cpu().numpy() for k, v in got.items()}
  t_gpu = time.perf_counter() - t0
  want = {}
  K = getattr(synth, cfg["K"])
  if "vsd" in errs:
    frames = d["frames"].cpu().numpy()
    want["vsd"], mssd_o, mspd_o = oracle.bop19_batch(
        objs, h["obj"], h["pe"], h["pg"], h["frame_idx"], frames, h["cam"], DELTA, TAUS,
        np.array([objs[o]["diameter"] for o in h["obj"]]))
    if "mssd" in errs:
      want["mssd"], want["mspd"] = mssd_o, mspd_o
    if c == 3 and png_src[0] is None:
      png_src[0] = frames[:24]
  elif "mssd" in errs:
    want["mssd"] = np.array([oracle.mssd(objs[o]["pts"], objs[o]["syms"], h["pe"][i],
                                         h["pg"][i]) for i, o in enumerate(h["obj"])])
    want["mspd"] = np.array([oracle.mspd(objs[o]["pts"], objs[o]["syms"], h["pe"][i],
                                         h["pg"][i], K) for i, o in enumerate(h["obj"])])
  if "add" in errs:
    want["add"] = np.array([oracle.add(objs[o]["pts"], h["pe"][i], h["pg"][i])
                            for i, o in enumerate(h["obj"])])
    want["adi"] = np.array([oracle.adi(objs[o]["pts"], h["pe"][i], h["pg"][i])
                            for i, o in enumerate(h["obj"])])
  row = {"tuples": int(n), "W": W, "H": H}
  for k in got:
    if k == "vsd":
      same = int((got[k] == want[k]).all(1).sum())
      row["vsd_rows_bit_identical"] = same
      ok &= same == n
    else:
      mab, mrel = _max_diff(got[k], want[k])
      row[k] = {"max_abs": mab, "max_rel": mrel}
      ok &= mab < PARITY_TOL
  row["s"] = round(time.perf_counter() - t0, 2)
  row["gpu_s"] = round(t_gpu, 2)
  res[str(c)] = row
  del ev, d
  return ok


def png_check(frames, torch):
  """Test-depth frames (integer mm) written as 16-bit PNGs by Pillow at zlib
  levels 0-9, decoded on the GPU (depth_gpu.DepthDecoder -> kern_png.hip) and
  compared bit for bit with Pillow's decode x the depth scale (inout.py:39-46,
  eval_calc_errors.py:242-243)."""
  import shutil
  import tempfile

  from PIL import Image

  from bop_toolkit_amd import depth_gpu
  tmp = tempfile.mkdtemp(prefix="bopx_bench_png_")
  try:
    q = np.clip(np.round(frames), 0, 65535).astype(np.uint16)
    n, Hh, Ww = q.shape
    paths, scales = [], []
    for i in range(n):
      path = os.path.join(tmp, "%06d.png" % i)
      Image.fromarray(q[i]).save(path, compress_level=i % 10)
      paths.append(path)
      scales.append(0.1 if i % 2 else 1.0)
    dec = depth_gpu.DepthDecoder(0)
    got = dec.load(paths, scales, Hh, Ww, torch).cpu().numpy()
    want = np.stack([np.asarray(Image.open(p_)).astype(np.float32) * np.float32(s_)
                     for p_, s_ in zip(paths, scales)])
    same = int(sum(np.array_equal(got[i], want[i]) for i in range(n)))
    return {"frames": n, "size": [Ww, Hh], "bit_identical": same,
            "device_decoded": n - int(dec.last_host), "zlib_levels": "0-9"}
  finally:
    shutil.rmtree(tmp, ignore_errors=True)


def cpu_baseline_point(objs, d, n):
  """configs[0] on the host: the oracle's ADD and brute-force ADI (C restatement
  of pose_error.py:147-184), one tuple after the other on one core."""
  from oracle import oracle
  h = d["host"]
  t0 = time.perf_counter()
  for i in range(n):
    pts = objs[h["obj"][i]]["pts"]
    oracle.add(pts, h["pe"][i], h["pg"][i])
    oracle.adi(pts, h["pe"][i], h["pg"][i])
  dt = time.perf_counter() - t0
  return {"value": n / dt, "unit": "tuples/s", "cores": 1, "kind": "port",
          "sample": "all %d tuples, ADD + ADI, %.2f s; oracle/bopx_oracle.c" % (n, dt)}


def main():
  args = parse()
  import torch
  import torch.distributed as dist

  # BOPX_DIST_BACKEND=gloo: rehearsal of the multi-rank flow with several ranks
  # on one GPU (host collectives); the measured configuration is RCCL, one GPU per rank.
  backend = os.environ.get("BOPX_DIST_BACKEND", "nccl")
  rw = world_of(args)
  if rw is None:  # --gpus N without torchrun: this process only launches the ranks
    # (device_count() does not initialise the GPU on this image)
    if backend == "nccl" and torch.cuda.device_count() < args.gpus:
      raise SystemExit("bench.py --gpus %d: only %d GPUs visible (RCCL needs one per rank)" %
                       (args.gpus, torch.cuda.device_count()))
    sys.exit(launch_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], args.gpus))
  rank, world, local = rw
  if backend == "gloo":
    local %= torch.cuda.device_count()
  torch.cuda.set_device(local)
  if world > 1:
    # a rank that dies leaves the others in a collective: bounded, so they fail
    # loudly (RCCL / gloo timeout error) instead of hanging to the caller's limit
    from datetime import timedelta
    tmo = timedelta(seconds=float(os.environ.get("BOPX_DIST_TIMEOUT_S", "300")))
    if backend == "nccl":
      dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
    else:
      dist.init_process_group(backend, timeout=tmo)
  from bop_toolkit_amd import shard
  from bop_toolkit_amd.batch import BatchEvaluator
  ev = BatchEvaluator(local)
  objs = build_objects(ev, args, torch)
  multi = "multi" in args.cfg
  n, d = (build_workload_multi if multi else build_workload)(ev, objs, args, rank, world, torch)
  meta = os.environ.get("BOPX_BENCH_META")  # tools/pmc.sh: what the counters measured
  if meta and rank == 0:
    with open(meta, "w") as f:
      json.dump({"lib_sha256": lib_digest(), "code_sha256": code_digests(),
                 "workload": workload_key(args, n)}, f)

  out_vsd = torch.empty((n, N_TAU), dtype=torch.float64, device=ev.device)
  out_mssd = torch.empty(n, dtype=torch.float64, device=ev.device)
  out_mspd = torch.empty(n, dtype=torch.float64, device=ev.device)
  rows = torch.empty((n, N_TAU + 2), dtype=torch.float64, device=ev.device)
  gids = d["gid"]
  ktime = {k: 0.0 for k in args.cfg["errors"]}
  marks = []  # per timed step: HIP events bracketing each kernel on the launch stream

  # MSSD / MSPD on a second stream: they fill the CUs k_vsd leaves idle
  # (its tail, LDS-bound residency) instead of queueing behind it.
  side = torch.cuda.Stream(device=ev.device) if os.environ.get("BOPX_BENCH_OVERLAP") else None

  # HIP events of every timed step, created before the timed region (event
  # creation is a runtime call per event; only record() runs inside it)
  pool = [{k: [torch.cuda.Event(enable_timing=True) for _ in range(2)] for k in ktime}
          for _ in range(args.steps)]

  def step(timed):
    e = pool[len(marks)] if timed else None
    rd = d.get("renders")
    run = {
        "vsd": (lambda: ev.vsd_shared(rd["slots"], rd["pose"], rd["frame_idx"], rd["est"],
                                      rd["gt"], d["frames"], d["cam"], DELTA, TAUS,
                                      d["diameters"], out=out_vsd)) if rd else
               (lambda: ev.vsd(d["slots"], d["pose_est"], d["pose_gt"], d["frame_idx"],
                               d["frames"], d["cam"], DELTA, TAUS, d["diameters"], out=out_vsd)),
        "mssd": lambda: ev.mssd(d["slots"], d["pose_est"], d["pose_gt"], out=out_mssd),
        "mspd": lambda: ev.mspd(d["slots"], d["pose_est"], d["pose_gt"], d["K"], out=out_mspd),
        "add": lambda: ev.add(d["slots"], d["pose_est"], d["pose_gt"], out=out_mssd),
        "adi": lambda: ev.adi(d["slots"], d["pose_est"], d["pose_gt"], out=out_mspd)}
    main = torch.cuda.current_stream(ev.device)
    if side is not None:
      side.wait_stream(main)  # previous step's rows consumed before they are rewritten
    for k in ktime:
      with torch.cuda.stream(side if side is not None and k != "vsd" else main):
        if e: e[k][0].record()
        run[k]()
        if e: e[k][1].record()
    if side is not None:
      main.wait_stream(side)
    if e: marks.append(e)
    if world > 1:
      rows[:, :N_TAU] = out_vsd
      rows[:, N_TAU] = out_mssd
      rows[:, N_TAU + 1] = out_mspd
      # per-tuple error rows -> rank 0, ordered by global tuple id (RCCL)
      if backend == "nccl":
        shard.gather_rows(rows, gids, d["n_total"], counts=d["counts"])
      else:
        shard.gather_rows(rows.cpu(), gids.cpu(), d["n_total"], counts=d["counts"])

  for _ in range(args.warmup):
    step(False)
  torch.cuda.synchronize()
  if world > 1:
    dist.barrier()
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for _ in range(args.steps):
    step(True)
  torch.cuda.synchronize()
  if world > 1:
    dist.barrier()
  torch.cuda.synchronize()
  elapsed = time.perf_counter() - t0
  for e in marks:
    for k in ktime:
      ktime[k] += e[k][0].elapsed_time(e[k][1]) * 1e-3
  if world > 1:
    tt = torch.tensor([elapsed], dtype=torch.float64,
                      device=ev.device if backend == "nccl" else "cpu")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt.item())

  fused_ms = None
  if multi:  # the same tuples through the fused per-tuple k_vsd, for comparison
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ref = ev.vsd(d["slots"], d["pose_est"], d["pose_gt"], d["frame_idx"], d["frames"], d["cam"],
                 DELTA, TAUS, d["diameters"])
    torch.cuda.synchronize()
    e0.record()
    for _ in range(max(1, args.steps // 2)):
      ev.vsd(d["slots"], d["pose_est"], d["pose_gt"], d["frame_idx"], d["frames"], d["cam"],
             DELTA, TAUS, d["diameters"], out=ref)
    e1.record()
    torch.cuda.synchronize()
    fused_ms = e0.elapsed_time(e1) / max(1, args.steps // 2)
    if not torch.equal(ref, out_vsd):
      raise RuntimeError("shared-render VSD differs from the fused kernel")
  if rank == 0:
    steps = args.steps
    total = d["n_total"] * steps
    from bop_toolkit_amd import synth
    cost = algorithmic_cost(objs, d["host"], n, getattr(synth, args.cfg["K"]))
    kt = {k: v / steps for k, v in ktime.items()}
    roof = None
    kernels = {}
    if kt:
      for k in kt:
        b, f32, f64 = cost[k]
        t_valu = f64 / (FP64_PEAK_TF * 1e12) + f32 / (FP32_PEAK_TF * 1e12)
        kernels[k] = {"ms": kt[k] * 1e3, "alg_GBps": b / kt[k] / 1e9}
        if k in ("mssd", "mspd"):
          # symmetry pruning (kern_pose.hip) skips (vertex, symmetry) pairs that
          # cannot change the minimum; SURVEY §8d counts every pair
          # not a roofline fraction: the ratio of the exhaustive sweep's VALU
          # roof time to the measured (pruned) time, i.e. a speed-up over an
          # ideal exhaustive kernel; the pruned sweep's own work is not counted
          kernels[k]["exhaustive_roof_speedup"] = {
              "value": round(t_valu / kt[k], 4), "unit": "x",
              "note": "SURVEY §8d fp64 roof time of the exhaustive (vertex, symmetry) sweep / "
                      "measured pruned kernel time"}
        else:
          kernels[k]["valu_roof_frac"] = t_valu / kt[k]
      dom = max(kt, key=kt.get)
      b, f32, f64 = cost[dom]
      ach = b / kt[dom] / 1e9
      t_valu = f64 / (FP64_PEAK_TF * 1e12) + f32 / (FP32_PEAK_TF * 1e12)
      # PMC bytes per launch, only from a summary of this library build on this
      # launch's workload (tools/pmc.sh records both), else null
      traffic = load_traffic(dom, args, n) if world == 1 else None
      roof = {"bound": "hbm", "achieved": round(ach, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "frac": round(ach / HBM_PEAK_GBS, 6), "traffic": traffic,
              "kernel": {"vsd": "k_vsd", "mssd": "k_sym_error<MSSD>", "mspd": "k_sym_error<MSPD>",
                         "add": "k_mean_error<ADD>", "adi": "k_adi"}[dom],
              "binding": {"roof": "valu", "frac": round(t_valu / kt[dom], 4),
                          "note": "VALU-bound by SURVEY.md §8d flop/byte; fp64 %.1f TF + "
                                  "fp32 %.1f TF peaks" % (FP64_PEAK_TF, FP32_PEAK_TF)}}
    cpu = None
    if world == 1 and not args.no_cpu_baseline and len(args.cfg["errors"]) == 3:
      cpu = cpu_baseline(objs, d, n, args.cpu_seconds, (out_vsd, out_mssd, out_mspd))
    elif world == 1 and not args.no_cpu_baseline and args.cfg["errors"] == ("add", "adi"):
      cpu = cpu_baseline_point(objs, d, n)
    parity = None
    if world == 1 and not args.no_parity and not args.no_cpu_baseline:
      # configurations this run already checked against the oracle (cpu_baseline.check)
      done = (args.config,) if cpu is not None and "check" in cpu else ()
      parity = parity_leg(args, torch, skip=done, png_frames=d["frames"][:24].cpu().numpy())
    e2e_images = args.e2e_images
    if e2e_images is None:
      # the metric's whole job as a dataset on disk (16,667 images = 100,002 tuples)
      e2e_images = 16667 if args.config == 3 and world == 1 and "multi" not in args.cfg else 0
    e2e = e2e_run(e2e_images, args.seed) if e2e_images > 0 and world == 1 else None
    line = {
        "metric": "pose-error tuples/sec (%s) at %dx%d, ~%dk-vert meshes" % (
            "+".join(e.upper() for e in args.cfg["errors"]), W, H,
            round(len(objs[0]["pts"]) / 1000)),
        "value": total / elapsed, "unit": "tuples/s", "n_gpus": world, "steps": steps,
        "warmup": args.warmup, "ms_per_step": elapsed / steps * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64+f32", "data": "synthetic",
        "config": {"workload": "%s, %d objs V=%d F=%d S in {%s}, %dx%d %s, %d tuples" % (
                                   args.cfg["what"], args.objects, len(objs[0]["pts"]),
                                   len(objs[0]["faces"]),
                                   ",".join(map(str, sorted(set(
                                       len(o["syms"]) for o in objs)))), W, H,
                                   args.cfg["K"].split("_")[0], d["n_total"]),
                   "global_batch": d["n_total"],
                   "parallelism": "image-sharded x%d (LPT)" % world,
                   "tuples_rank0": n,
                   "roi_mean_px": round(cost["roi_mean"], 1),
                   **({"axes_scale": args.axes_scale} if args.axes_scale != 1.0 else {})},
        "roofline": roof, "kernels": kernels, "cpu_baseline": cpu, "parity": parity, "e2e": e2e}
    if multi:
      rd = d["renders"]
      if roof is not None and roof["kernel"] == "k_vsd":
        roof["kernel"] = "k_vsd (render mode) + k_vsd_pair"
        roof["note"] = "algorithmic bytes / flops of the per-tuple model (two renders each)"
      line["config"]["renders"] = rd["n"]
      line["kernels"]["vsd_fused_per_tuple"] = {"ms": fused_ms,
                                                "renders": 2 * n,
                                                "note": "same tuples, two renders each (k_vsd)"}
    print(json.dumps(line), flush=True)
  if world > 1:
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
  main()
