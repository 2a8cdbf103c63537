"""Multi-GPU partitioning of an error-evaluation job.

Tuples are independent (no cross-tuple term in pose_error.*), so the job is
sharded with no data-path collective: images are assigned to ranks by LPT
(longest-processing-time-first) bin packing on an estimated cost, each rank
evaluates its images' tuples on its own GPU, and the per-tuple error rows are
gathered to rank 0 once at the end (an RCCL gather over xGMI on GPUs, gloo on CPU).
Images, not scenes, are the unit: LM-O and ITODD have a single test scene
(dataset_params.py:345,447-451), so scene sharding cannot balance 8 GPUs.

The gathered table is re-ordered by global tuple id, so it is bitwise
identical to a single-GPU run.
"""
import heapq

import numpy as np


def tuple_cost(nv, nf, ns, roi_px):
  """Relative cost of one BOP19 tuple (VSD + MSSD + MSPD), from the per-tuple
  flop model of SURVEY.md §8d: VSD 40V + 60F + 92 ROI, MSSD V(18 + 28S),
  MSPD V(20 + 27S)."""
  nv, nf, ns, roi_px = (np.asarray(x, np.float64) for x in (nv, nf, ns, roi_px))
  return 40 * nv + 60 * nf + 92 * roi_px + nv * (38 + 55 * ns)


def error_cost(error_type, nv, nf, ns, roi_px):
  """Relative cost of one tuple of one error type (SURVEY.md §8d flop model):
  VSD 40V + 60F + 92 ROI, CUS 40V + 60F + 34 ROI, MSSD V(18 + 28S), MSPD
  V(20 + 27S), ADD / PROJ 46V, ADI 36V + 9V^2 (AD: the ADD cost; the caller
  does not know which objects are symmetric here, a constant factor at most)."""
  nv, nf, ns, roi_px = (np.asarray(x, np.float64) for x in (nv, nf, ns, roi_px))
  if error_type == "vsd":
    return 40 * nv + 60 * nf + 92 * roi_px
  if error_type == "cus":
    return 40 * nv + 60 * nf + 34 * roi_px
  if error_type == "mssd":
    return nv * (18 + 28 * ns)
  if error_type == "mspd":
    return nv * (20 + 27 * ns)
  if error_type == "adi":
    return 36 * nv + 9 * nv * nv
  return 46 * nv + 0 * roi_px


def roi_pixels(lo, hi, poses, K, width, height):
  """SURVEY.md §8d ROI of each tuple: the union over its poses of the clipped
  screen bbox of the projected 8 corners of the model's bounding box (the whole
  image if a corner is behind the camera). lo, hi: n x 3 model bbox corners;
  poses: list of n x 12 [R | t] arrays; K: 3 x 3 or n x 3 x 3."""
  lo, hi = np.asarray(lo, np.float64), np.asarray(hi, np.float64)
  n = len(lo)
  K = np.broadcast_to(np.asarray(K, np.float64), (n, 3, 3))
  corners = np.stack([np.where(np.array([(k >> a) & 1 for a in range(3)]) == 1, hi, lo)
                      for k in range(8)], 1)  # n x 8 x 3
  x0 = np.full(n, np.inf)
  y0 = np.full(n, np.inf)
  x1 = np.full(n, -np.inf)
  y1 = np.full(n, -np.inf)
  full = np.zeros(n, bool)
  for p in poses:
    p = np.asarray(p, np.float64)
    R = p[:, :9].reshape(n, 3, 3)
    X = np.einsum("nij,nkj->nki", R, corners) + p[:, None, 9:]
    full |= (X[..., 2] <= 0).any(1)
    Z = np.where(X[..., 2] > 0, X[..., 2], 1.0)
    u = K[:, 0, 0, None] * X[..., 0] / Z + K[:, 0, 2, None]
    v = K[:, 1, 1, None] * X[..., 1] / Z + K[:, 1, 2, None]
    x0 = np.minimum(x0, u.min(1))
    x1 = np.maximum(x1, u.max(1))
    y0 = np.minimum(y0, v.min(1))
    y1 = np.maximum(y1, v.max(1))
  with np.errstate(invalid="ignore"):
    w = np.clip(np.floor(x1), -1, width - 1) - np.clip(np.ceil(x0), 0, width) + 1
    h = np.clip(np.floor(y1), -1, height - 1) - np.clip(np.ceil(y0), 0, height) + 1
  area = np.maximum(np.nan_to_num(w), 0) * np.maximum(np.nan_to_num(h), 0)
  area[full] = width * height
  return area


def lpt_shard(costs, world):
  """Assign items (images) to `world` ranks, heaviest first, each to the
  currently lightest rank (ties -> lowest rank). Returns a list of index
  arrays, one per rank, each sorted ascending."""
  costs = np.asarray(costs, np.float64)
  order = np.argsort(-costs, kind="stable")
  heap = [(0.0, r) for r in range(world)]
  heapq.heapify(heap)
  parts = [[] for _ in range(world)]
  for i in order:
    load, r = heapq.heappop(heap)
    parts[r].append(int(i))
    heapq.heappush(heap, (load + float(costs[i]), r))
  return [np.array(sorted(p), dtype=np.int64) for p in parts]


def image_costs(frame_of_tuple, per_tuple_cost, n_images):
  """Sum per-tuple costs into per-image costs."""
  return np.bincount(np.asarray(frame_of_tuple), weights=per_tuple_cost, minlength=n_images)


def gather_rows(rows, ids, n_total, group=None, counts=None):
  """Gather per-tuple rows from every rank to rank 0.

  rows: [n_local, C] float64 tensor on this rank's device (or CPU for gloo);
  ids:  [n_local] int64 tensor of global tuple ids.
  counts: the n_local of every rank when the caller knows them (a fixed shard
  per rank, e.g. bench.py); otherwise one all_gather of the counts first.
  Returns the [n_total, C] table ordered by global id on rank 0, None elsewhere.
  One padded gather of [id | row] blocks to rank 0, scattered by id there.
  """
  import torch
  import torch.distributed as dist
  world = dist.get_world_size(group)
  rank = dist.get_rank(group)
  dev = rows.device
  if counts is None:
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=dev)
    cl = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(cl, n, group=group)
    counts = [int(c.item()) for c in cl]
  counts = [int(c) for c in counts]
  if len(counts) != world or counts[rank] != rows.shape[0]:
    raise ValueError("gather_rows: counts %r do not match this rank's %d rows"
                     % (counts, rows.shape[0]))
  width = rows.shape[1] + 1
  pad = max(counts)
  block = torch.zeros((pad, width), dtype=torch.float64, device=dev)
  block[:rows.shape[0], 0] = ids.to(torch.float64)
  block[:rows.shape[0], 1:] = rows
  # a real gather to rank 0 (RCCL: point-to-point sends over xGMI; gloo: host
  # collectives): only the root receives the table
  out = torch.empty((world * pad, width), dtype=torch.float64, device=dev) if rank == 0 else None
  if dev.type == "cuda" and dist.get_backend(group) != "nccl":  # gloo: staged through the host
    host = out.cpu() if out is not None else None
    dist.gather(block.cpu(), list(host.view(world, pad, width).unbind(0)) if rank == 0 else None,
                dst=0, group=group)
    if rank == 0:
      out.copy_(host)
  else:
    dist.gather(block, list(out.view(world, pad, width).unbind(0)) if rank == 0 else None, dst=0,
                group=group)
  if rank != 0:
    return None
  if pad * world != sum(counts):  # drop the padding rows
    keep = torch.cat([torch.arange(r * pad, r * pad + c, device=dev)
                      for r, c in enumerate(counts)])
    out = out.index_select(0, keep)
  gid = out[:, 0].to(torch.int64)
  if out.shape[0] != n_total or not bool(
      (torch.bincount(gid, minlength=n_total)[:n_total] == 1).all()):
    raise RuntimeError("gather_rows: tuple ids are not a permutation of 0..%d" % (n_total - 1))
  table = torch.empty((n_total, rows.shape[1]), dtype=torch.float64, device=dev)
  table[gid] = out[:, 1:]
  return table


def init_from_env():
  """One process per GPU under torchrun (RANK / WORLD_SIZE / LOCAL_RANK):
  bind the local GPU and join the RCCL group. Returns (rank, world, local)."""
  import os
  world = int(os.environ.get("WORLD_SIZE", 1))
  local = int(os.environ.get("LOCAL_RANK", os.environ.get("BOPX_DEVICE", 0)))
  if world <= 1:
    return 0, 1, local
  import torch
  import torch.distributed as dist
  # BOPX_DIST_BACKEND=gloo: host collectives, ranks may share a GPU (rehearsal
  # of the multi-rank flow on a one-GPU machine); default RCCL, one GPU per rank.
  backend = os.environ.get("BOPX_DIST_BACKEND", "nccl")
  if backend == "gloo":
    local %= max(1, torch.cuda.device_count())
  torch.cuda.set_device(local)
  if not dist.is_initialized():
    if backend == "nccl":
      dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
      dist.init_process_group(backend)
  return dist.get_rank(), world, local
