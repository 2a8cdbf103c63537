"""Multi-GPU partitioning of an error-evaluation job.

Tuples are independent (no cross-tuple term in pose_error.*), so the job is
sharded with no data-path collective: images are assigned to ranks by LPT
(longest-processing-time-first) bin packing on an estimated cost, each rank
evaluates its images' tuples on its own GPU, and the per-tuple error rows are
gathered to rank 0 once at the end (RCCL over xGMI on GPUs, gloo on CPU).
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
  One padded all_gather of [id | row] blocks, scattered by id on rank 0.
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
  out = torch.empty((world * pad, width), dtype=torch.float64, device=dev)
  if dev.type == "cuda" and dist.get_backend(group) == "nccl":  # RCCL: one contiguous all-gather
    dist.all_gather_into_tensor(out, block, group=group)
  else:  # gloo (host collectives; device rows are staged through host memory)
    host = out.cpu() if dev.type == "cuda" else out
    dist.all_gather(list(host.view(world, pad, width).unbind(0)), block.cpu(), group=group)
    if host is not out:
      out.copy_(host)
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
