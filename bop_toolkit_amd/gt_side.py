"""GT-side counterparts of scripts/calc_gt_info.py and scripts/calc_gt_masks.py
(SURVEY.md §8f-3): the same raster + bop19 visibility as VSD, one fused
launch per batch of GT instances (k_vsd GT-info mode) instead of one OpenGL
render and three full-frame NumPy passes per instance.

    python -m bop_toolkit_amd.gt_side info  --dataset lmo --dataset_split test
    python -m bop_toolkit_amd.gt_side masks --dataset lmo --dataset_split test

Outputs are the reference's: scene_gt_info.json (px_count_all /_valid /_visib,
visib_fract, bbox_obj, bbox_visib per GT, calc_gt_info.py:113-168) and the
mask / mask_visib PNGs (0/255, calc_gt_masks.py:104-125). calc_gt_info uses
a canvas three times the image with the image in its centre, so silhouettes of
objects truncated by the image border are counted whole (calc_gt_info.py:66-73,
104-107); calc_gt_masks renders at image size. The reference's
calc_gt_masks.py processes a hard-coded `scene_ids = [0]` (calc_gt_masks.py:56);
here every present scene is processed unless --scene_ids narrows it.
"""
import argparse
import os

import numpy as np

from . import dataset_params, inout, misc

INFO_KEYS = ("px_count_all", "px_count_valid", "px_count_visib", "visib_fract", "bbox_obj",
             "bbox_visib")


def info_from_row(row):
  """One scene_gt_info entry from a k_vsd GT-info row."""
  n_all, n_visib, n_valid = int(row[0]), int(row[1]), int(row[10])
  bb = [int(v) for v in row[2:10]]
  bbox_obj, bbox_visib = [-1, -1, -1, -1], [-1, -1, -1, -1]
  if n_visib > 0:  # both boxes only when something is visible (calc_gt_info.py:139-151)
    bbox_obj = [bb[0], bb[1], bb[2] - bb[0], bb[3] - bb[1]]
    bbox_visib = [bb[4], bb[5], bb[6] - bb[4], bb[7] - bb[5]]
  return {"px_count_all": n_all, "px_count_valid": n_valid, "px_count_visib": n_visib,
          "visib_fract": float(n_visib / float(n_all) if n_all > 0 else 0.0),
          "bbox_obj": bbox_obj, "bbox_visib": bbox_visib}


_INFO_FMT = ('{"bbox_obj": [%d, %d, %d, %d], "bbox_visib": [%d, %d, %d, %d], "px_count_all": %d, '
             '"px_count_valid": %d, "px_count_visib": %d, "visib_fract": %r}')


def save_scene_gt_info(path, rows):
  """inout.save_json(path, {im_id: [info_from_row(r) for r in lst]}) for
  rows = {im_id: [row, ...]}, byte for byte, formatted straight from the rows
  (sorted keys, one image per line; visib_fract by float repr like the JSON
  encoder)."""
  ims = sorted(rows)
  flat = [r for im in ims for r in rows[im]]
  lines = []
  if flat:
    a = np.asarray(flat, np.float64).reshape(-1, 11)
    ints = a.astype(np.int64)
    n_all, n_vis = ints[:, 0], ints[:, 1]
    fr = np.where(n_all > 0, n_vis / np.where(n_all > 0, n_all, 1), 0.0)
    bb = ints[:, 2:10].copy()
    bb[:, 2] -= bb[:, 0]
    bb[:, 3] -= bb[:, 1]
    bb[:, 6] -= bb[:, 4]
    bb[:, 7] -= bb[:, 5]
    bb[n_vis <= 0] = -1  # both boxes only when something is visible
    vals = np.concatenate([bb, n_all[:, None], ints[:, 10:11], n_vis[:, None]], 1).tolist()
    recs = [_INFO_FMT % (tuple(v) + (f,)) for v, f in zip(vals, fr.tolist())]
  k = 0
  for im in ims:
    n = len(rows[im])
    lines.append('  "%d": [%s]' % (im, ", ".join(recs[k:k + n])))
    k += n
  with open(path, "w") as f:
    f.write("{\n" + ",\n".join(lines) + ("\n}" if lines else "}"))


def _cached(loader, path):
  """loader(path) through the evaluation's parse cache (the same objects for
  every pass of this process; read-only)."""
  from .eval_calc_errors import cached_load
  return cached_load(loader, path)


def _depth_path(dp_split, scene_id, im_id):
  path = dp_split["depth_tpath"].format(scene_id=scene_id, im_id=im_id)
  return path if os.path.exists(path) else path.replace(".tif", ".png")


def _scene_gt(path):
  """A scene's GT: the native reader's inout.GTLists (no Python JSON parse
  under the GIL on the prefetch thread), or load_scene_gt's dict when it
  declines the file (eval_calc_errors.scene_gt_arrays)."""
  from .eval_calc_errors import scene_gt_arrays
  return scene_gt_arrays(path)


def _gt_count(scene_gt, im_id):
  if isinstance(scene_gt, inout.GTLists):
    a, b = scene_gt.rows(im_id)
    return b - a
  return len(scene_gt[im_id])


def _gt_ims(scene_gt):
  return sorted(scene_gt.index if isinstance(scene_gt, inout.GTLists) else scene_gt.keys())


def my_images(scene_gt, rank, world):
  """This rank's image ids of a scene (LPT on the GT count per image)."""
  from . import shard
  im_ids = _gt_ims(scene_gt)
  if world == 1:
    return im_ids
  part = shard.lpt_shard([_gt_count(scene_gt, i) + 1 for i in im_ids], world)[rank]
  return [im_ids[k] for k in part]


_PINNED = [None, None]  # page-locked depth staging buffers (scene_stats)


def scene_stats(ev, torch, dp_split, scene_id, delta, canvas_scale, masks, im_batch=None,
                rank=0, world=1, frames_all=None):
  """Per image id: list of (row, masks or None) per GT instance, in GT order;
  images are evaluated in batches of im_batch frames (default: 128 when the
  frames are decoded here or mask planes come back; the whole scene in one
  launch when its frames are resident and only the rows are read). With
  world > 1 only this rank's images (my_images) are evaluated. frames_all: the
  test depth of those images already on the device (SceneDepthPrefetch), else
  it is decoded here on the host, a batch ahead."""
  from . import runtime
  scene_camera = _cached(inout.load_scene_camera,
                         dp_split["scene_camera_tpath"].format(scene_id=scene_id))
  scene_gt = _scene_gt(dp_split["scene_gt_tpath"].format(scene_id=scene_id))
  lists = isinstance(scene_gt, inout.GTLists)
  im_ids = my_images(scene_gt, rank, world)
  if im_batch is None:
    im_batch = max(1, len(im_ids)) if frames_all is not None and not masks else 128
  res = {}
  dev = ev.device
  W, H = dp_split["im_size"]

  def load(ims, slot):
    # test depth in mm (float32 in place, calc_gt_info.py:99-100), decoded into
    # a page-locked buffer while the previous batch runs; two buffers used in
    # turn across batches and scenes (batch bi's upload has completed when
    # bi + 2 is decoded: its rows were read back in between)
    paths = [_depth_path(dp_split, scene_id, im_id) for im_id in ims]
    scales = [scene_camera[im_id]["depth_scale"] for im_id in ims]
    if torch.cuda.is_available():
      need = len(ims) * H * W
      if _PINNED[slot] is None or _PINNED[slot].numel() < need:
        _PINNED[slot] = None
        _PINNED[slot] = torch.empty(max(need, im_batch * H * W), dtype=torch.float32,
                                    pin_memory=True)
      buf = _PINNED[slot][:need].view(len(ims), H, W)
      try:
        inout.load_depths(paths, scales=scales, out=buf.numpy())
        return buf
      except ValueError:
        pass  # a frame of another size
    return np.stack(inout.load_depths(paths, scales=scales))

  from concurrent.futures import ThreadPoolExecutor
  batches = [im_ids[i0:i0 + im_batch] for i0 in range(0, len(im_ids), im_batch)]
  if frames_all is not None and len(frames_all) != len(im_ids):
    raise ValueError("frames_all holds %d frames for %d images" % (len(frames_all), len(im_ids)))
  with ThreadPoolExecutor(1) as ahead:
    nxt = None
    if batches and frames_all is None:
      nxt = ahead.submit(load, batches[0], 0)
    for bi, ims in enumerate(batches):
      if frames_all is not None:
        frames = frames_all[bi * im_batch:bi * im_batch + len(ims)]
      else:
        frames = nxt.result()
        if bi + 1 < len(batches):
          nxt = ahead.submit(load, batches[bi + 1], (bi + 1) & 1)
      cam, obj, Rs, ts, fidx, owner, rws = [], [], [], [], [], [], []
      for k, im_id in enumerate(ims):
        K = scene_camera[im_id]["cam_K"]
        cam.append((K[0, 0], K[1, 1], K[0, 2], K[1, 2]))
        if lists:
          a, b = scene_gt.rows(im_id)
          obj.extend(scene_gt.obj[a:b].tolist())
          rws.extend(range(a, b))
          fidx.extend([k] * (b - a))
          owner.extend([im_id] * (b - a))
        else:
          for gt in scene_gt[im_id]:
            obj.append(gt["obj_id"])
            Rs.append(gt["cam_R_m2c"])
            ts.append(gt["cam_t_m2c"])
            fidx.append(k)
            owner.append(im_id)
        res[im_id] = []
      if not obj:
        continue
      # [R row-major | t] per GT, float64
      if lists:
        rws = np.asarray(rws, np.int64)
        pose = np.concatenate([scene_gt.fields["cam_R_m2c"][rws],
                               scene_gt.fields["cam_t_m2c"][rws]], 1)
      else:
        pose = np.concatenate([np.asarray(Rs, np.float64).reshape(-1, 9),
                               np.asarray(ts, np.float64).reshape(-1, 3)], 1)
      T = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
      d_frames = (frames.to(dev, non_blocking=True) if torch.is_tensor(frames)
                  else T(frames, torch.float32))
      rows, mk = ev.gt_info(ev.slots(obj), T(pose, torch.float64),
                            T(np.array(fidx, np.int32), torch.int32), d_frames,
                            T(np.array(cam), torch.float64), delta, canvas_scale, masks,
                            runtime.delta_flags(delta))
      rows = rows.cpu().numpy()
      mk = mk.cpu().numpy() if mk is not None else None
      for j, im_id in enumerate(owner):
        res[im_id].append((rows[j], None if mk is None else mk[j]))
  return res


def _setup(p):
  import torch
  from .batch import BatchEvaluator
  dp_split = dataset_params.get_split_params(p["datasets_path"], p["dataset"],
                                             p["dataset_split"], p["dataset_split_type"])
  dp_model = dataset_params.get_model_params(p["datasets_path"], p["dataset"],
                                             "cad" if p["dataset"] == "tless" else None)
  import os as _os
  ev = BatchEvaluator(int(_os.environ.get("LOCAL_RANK", p.get("device", 0))))
  misc.log("Initializing renderer...")
  for obj_id in dp_model["obj_ids"]:
    path = dp_model["model_tpath"].format(obj_id=obj_id)
    if os.path.exists(path):
      m = inout.load_ply(path)
      ev.add_object(obj_id, m["pts"], m.get("faces"))
  scene_ids = p.get("scene_ids") or dataset_params.get_present_scene_ids(dp_split)
  return torch, ev, dp_split, scene_ids


def _gather_info(torch, ev, stats, scene_gt, rank, world):
  """{im_id: [row]} of the whole scene on rank 0 (RCCL gather of the rows)."""
  if world == 1:
    return {im: [r for r, _ in lst] for im, lst in stats.items()}
  from . import shard
  ims = _gt_ims(scene_gt)
  first = np.cumsum([0] + [_gt_count(scene_gt, i) for i in ims])
  pos = {im: int(first[k]) for k, im in enumerate(ims)}
  ids, rows = [], []
  for im, lst in stats.items():
    for g, (r, _) in enumerate(lst):
      ids.append(pos[im] + g)
      rows.append(r)
  dev = ev.device
  table = shard.gather_rows(
      torch.as_tensor(np.array(rows, np.float64).reshape(-1, 11), device=dev),
      torch.as_tensor(np.array(ids, np.int64), device=dev), int(first[-1]))
  if rank != 0:
    return None
  table = table.cpu().numpy()
  return {im: [table[pos[im] + g] for g in range(_gt_count(scene_gt, im))] for im in ims}


class SceneDepthPrefetch:
  """The scenes' test depth decoded on the GPU (depth_gpu, kern_png.hip) ahead
  of use, consecutive scenes in shared launches (depth_gpu.GroupPrefetch, the
  VSD error pass's grouping: BOPX_DEPTH_GROUP_FRAMES): take(scene) returns the
  frames of this rank's images (my_images order) on the device, final for the
  current stream. None for a scene (host decoding in scene_stats) without a
  GPU, with BOPX_DEPTH_GPU=0, without a GT file, or when a frame of its group
  has another size."""

  def __init__(self, ev, torch, dp_split, rank, world, scene_ids=()):
    from . import depth_gpu
    from .eval_calc_errors import depth_group_sizes
    self.on = torch.cuda.is_available() and depth_gpu.enabled()
    self.groups = None
    g, first = depth_group_sizes()
    if not self.on or g <= 0 or not scene_ids:
      return
    dp = dp_split

    def paths(scene_id):
      path_gt = dp["scene_gt_tpath"].format(scene_id=scene_id)
      if not os.path.exists(path_gt):
        return [], []
      scene_camera = _cached(inout.load_scene_camera,
                             dp["scene_camera_tpath"].format(scene_id=scene_id))
      im_ids = my_images(_scene_gt(path_gt), rank, world)
      return ([_depth_path(dp, scene_id, i) for i in im_ids],
              [scene_camera[i]["depth_scale"] for i in im_ids])
    W, H = dp["im_size"]
    dev = ev.device
    self.groups = depth_gpu.GroupPrefetch(
        dev.index or 0, [(sid, (lambda sid=sid: paths(sid))) for sid in scene_ids], H, W, torch,
        torch.cuda.Stream(dev), torch.cuda.current_stream(dev), max_frames=g, first_frames=first,
        max_groups=3)

  def take(self, scene_id):
    if self.groups is None:
      return None
    try:
      return self.groups.get(scene_id)
    except ValueError:
      return None  # a frame of another size in its group: host decoding

  def close(self):
    if self.groups is not None:
      self.groups.close()


def calc_gt_info(p):
  """scene_gt_info.json of every scene (calc_gt_info.py:75-175); returns paths.
  Under torchrun the images of each scene are split over the GPUs and rank 0
  writes the file."""
  from . import shard
  rank, world, _ = shard.init_from_env()
  torch, ev, dp_split, scene_ids = _setup(p)
  written = []
  ahead = SceneDepthPrefetch(ev, torch, dp_split, rank, world, scene_ids)
  try:
    for scene_id in scene_ids:
      misc.log("Calculating GT info - dataset: {} ({}, {}), scene: {}".format(
          p["dataset"], p["dataset_split"], p["dataset_split_type"], scene_id))
      frames = ahead.take(scene_id)
      stats = scene_stats(ev, torch, dp_split, scene_id, p["delta"], 3, False, rank=rank,
                          world=world, frames_all=frames)
      scene_gt = _scene_gt(dp_split["scene_gt_tpath"].format(scene_id=scene_id))
      rows = _gather_info(torch, ev, stats, scene_gt, rank, world)
      if rows is None:
        continue
      path = dp_split["scene_gt_info_tpath"].format(scene_id=scene_id)
      os.makedirs(os.path.dirname(path), exist_ok=True)
      save_scene_gt_info(path, rows)
      written.append(path)
  finally:
    ahead.close()
  return written


def calc_gt_masks(p):
  """mask / mask_visib PNGs of every GT instance (calc_gt_masks.py:58-125).
  Under torchrun every rank writes the masks of its own images."""
  from PIL import Image
  from . import shard
  rank, world, _ = shard.init_from_env()
  torch, ev, dp_split, scene_ids = _setup(p)
  written = []
  ahead = SceneDepthPrefetch(ev, torch, dp_split, rank, world, scene_ids)
  try:
    for scene_id in scene_ids:
      frames = ahead.take(scene_id)
      if not os.path.exists(dp_split["scene_gt_tpath"].format(scene_id=scene_id)):
        print("Skip scene {} (GT file not found).".format(scene_id))
        continue
      misc.log("Calculating masks - dataset: {} ({}, {}), scene: {}".format(
          p["dataset"], p["dataset_split"], p["dataset_split_type"], scene_id))
      stats = scene_stats(ev, torch, dp_split, scene_id, p["delta"], 1, True, rank=rank,
                          world=world, frames_all=frames)
      for im_id, lst in stats.items():
        for gt_id, (_, mk) in enumerate(lst):
          for plane, key in enumerate(("mask_tpath", "mask_visib_tpath")):
            path = dp_split[key].format(scene_id=scene_id, im_id=im_id, gt_id=gt_id)
            os.makedirs(os.path.dirname(path), exist_ok=True)
            Image.fromarray(mk[plane]).save(path)
            written.append(path)
  finally:
    ahead.close()
  return written


def parse_args(argv=None):
  ap = argparse.ArgumentParser()
  ap.add_argument("task", choices=["info", "masks"])
  ap.add_argument("--dataset", default="lmo")
  ap.add_argument("--dataset_split", default="test")
  ap.add_argument("--dataset_split_type", default=None)
  ap.add_argument("--delta", type=float, default=15)
  ap.add_argument("--renderer_type", default="hip")
  ap.add_argument("--datasets_path", default=os.environ.get("BOP_PATH", "/path/to/bop"))
  ap.add_argument("--scene_ids", default="")
  a = ap.parse_args(argv)
  delta = int(a.delta) if float(a.delta).is_integer() else a.delta  # reference: int 15
  p = {"dataset": a.dataset, "dataset_split": a.dataset_split,
       "dataset_split_type": a.dataset_split_type, "delta": delta,
       "renderer_type": a.renderer_type, "datasets_path": a.datasets_path,
       "scene_ids": [int(x) for x in a.scene_ids.split(",") if x]}
  return a.task, p


def main(argv=None):
  task, p = parse_args(argv)
  (calc_gt_info if task == "info" else calc_gt_masks)(p)


if __name__ == "__main__":
  main()
