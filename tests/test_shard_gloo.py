"""Multi-process sharding / gather on CPU (gloo, world sizes 2, 4 and 8): the
gathered table is bitwise identical to the single-process table (SURVEY.md
§8e), also when ranks get no images at all (4 test images over 8 ranks)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bop_toolkit_amd import shard


def _free_port():
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  p = s.getsockname()[1]
  s.close()
  return p


def test_lpt_balances_and_partitions():
  rng = np.random.default_rng(0)
  costs = rng.pareto(1.5, 500) + 1.0
  parts = shard.lpt_shard(costs, 8)
  allidx = np.sort(np.concatenate(parts))
  assert np.array_equal(allidx, np.arange(500))
  loads = np.array([costs[p].sum() for p in parts])
  assert loads.max() <= loads.mean() + costs.max()  # LPT bound
  assert shard.lpt_shard(costs, 8)[3].tolist() == parts[3].tolist()  # deterministic


def test_single_image_scene_still_shards():
  # LM-O: one test scene -> sharding by image must still use every rank
  costs = np.ones(200)
  parts = shard.lpt_shard(costs, 8)
  assert all(len(p) == 25 for p in parts)


def _worker(rank, world, port, n_img, out_path):
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  rng = np.random.default_rng(5)
  frame_of_tuple = np.repeat(np.arange(n_img), 6)
  cost = shard.tuple_cost(np.full(len(frame_of_tuple), 5002), 10000,
                          rng.integers(1, 9, len(frame_of_tuple)),
                          rng.uniform(1e4, 7e4, len(frame_of_tuple)))
  parts = shard.lpt_shard(shard.image_costs(frame_of_tuple, cost, n_img), world)
  mine = np.nonzero(np.isin(frame_of_tuple, parts[rank]))[0]
  # "evaluate": a deterministic function of the global tuple id
  full = np.sin(np.arange(len(frame_of_tuple))[:, None] * np.arange(1, 13)[None, :])
  rows = torch.from_numpy(full[mine])
  table = shard.gather_rows(rows, torch.from_numpy(mine), len(frame_of_tuple))
  # counts known up front (bench.py's fixed shards): no count exchange
  counts = [int(np.isin(frame_of_tuple, p).sum()) for p in parts]
  table2 = shard.gather_rows(rows, torch.from_numpy(mine), len(frame_of_tuple), counts=counts)
  if rank == 0:
    assert torch.equal(table, table2)
    np.save(out_path, table.numpy())
  dist.barrier()
  dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gather_bitwise_equals_single(tmp_path, world):
  out = str(tmp_path / "table.npy")
  n_img = 37
  mp.spawn(_worker, args=(world, _free_port(), n_img, out), nprocs=world, join=True)
  table = np.load(out)
  full = np.sin(np.arange(n_img * 6)[:, None] * np.arange(1, 13)[None, :])
  assert np.array_equal(table, full)


def _stub_rows(ev, torch_, p, dataset, dp_split, scene_camera, scene_id, recs, models_info,
               sym_ids, todo):
  """Stand-in for the GPU batch: a deterministic function of (record, gt)."""
  width = len(p["vsd_taus"]) if p["error_type"] == "vsd" else 1
  return torch.tensor([[ri * 1000.0 + gt_id + 0.1 * k for k in range(width)]
                       for ri, gt_id, _, _ in todo], dtype=torch.float64)


class _FakeEv:
  """The object table the caller's LPT cost model reads (BatchEvaluator.objects)
  without a GPU: sizes per object, bbox from models_info.json."""

  def __init__(self, info):
    import torch as _t
    self.device = _t.device("cpu")
    self.objects = {}
    for k, (obj_id, m) in enumerate(sorted(info.items())):
      lo = np.array([m["min_x"], m["min_y"], m["min_z"]])
      hi = lo + np.array([m["size_x"], m["size_y"], m["size_z"]])
      self.objects[obj_id] = {"nv": 1000 + 700 * k, "nf": 2000 + 1400 * k, "ns": 1 + k,
                              "bbox": (lo, hi)}


def _caller_errs(error_type="vsd", with_costs=False):
  from bop_toolkit_amd import dataset_params, eval_calc_errors as ece, inout
  e2e = os.path.join(os.path.dirname(__file__), "golden", "e2e")
  p = ece.parse_args(["--error_type", error_type, "--n_top", "-1", "--result_filenames",
                      "synth_lmo-test.csv", "--results_path", os.path.join(e2e, "results"),
                      "--datasets_path", os.path.join(e2e, "datasets")])
  dp_split = dataset_params.get_split_params(p["datasets_path"], "lmo", "test")
  dp_model = dataset_params.get_model_params(p["datasets_path"], "lmo", "eval")
  targets = inout.load_json(os.path.join(dp_split["base_path"], p["targets_filename"]))
  ests = inout.load_bop_results(os.path.join(p["results_path"], "synth_lmo-test.csv"))
  t_org, e_org = ece.organize(targets, ests)
  info = inout.load_json(dp_model["models_info_path"], keys_to_int=True)
  scene_gt = inout.load_scene_gt(dp_split["scene_gt_tpath"].format(scene_id=2))
  scene_camera = inout.load_scene_camera(dp_split["scene_camera_tpath"].format(scene_id=2))
  recs, _ = ece.scene_records(p, 2, t_org[2], e_org, scene_gt)
  ev = _FakeEv(info) if with_costs else None
  return ece.evaluate(ev, torch, p, "lmo", dp_split, scene_camera, 2, recs, info, set(),
                      batch_fn=_stub_rows)


def _caller_worker(rank, world, port, out_path, error_type, with_costs):
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  errs = _caller_errs(error_type, with_costs)
  if rank == 0:
    import json
    with open(out_path, "w") as f:
      json.dump([{str(k): v for k, v in e.items()} for e in errs], f)
  else:
    assert errs is None
  dist.barrier()
  dist.destroy_process_group()


@pytest.mark.parametrize("world,error_type,with_costs", [
    (2, "vsd", False), (2, "vsd", True), (4, "mssd", True), (8, "vsd", True),
    (8, "mssd", True)])
def test_caller_sharded_equals_single(tmp_path, world, error_type, with_costs):
  """eval_calc_errors.evaluate under gloo (images of the scene split by LPT on
  the SURVEY §8d tuple costs, rows gathered to rank 0) == the single-process
  result. World 8 > the 4 test images: some ranks evaluate nothing and still
  join the gather with zero rows."""
  import json
  out = str(tmp_path / "errs.json")
  mp.spawn(_caller_worker, args=(world, _free_port(), out, error_type, with_costs),
           nprocs=world, join=True)
  single = [{str(k): v for k, v in e.items()} for e in _caller_errs(error_type, with_costs)]
  assert json.load(open(out)) == single
  assert sum(v[0] != 1.0 and v[0] < 1e6 for e in single for v in e.values()) > 10


def test_caller_cost_model_shapes_the_shard():
  """todo_costs: VSD costs grow with the projected ROI, MSSD costs with V * S,
  and the LPT shard built from them covers every tuple exactly once."""
  from bop_toolkit_amd import dataset_params, eval_calc_errors as ece, inout
  e2e = os.path.join(os.path.dirname(__file__), "golden", "e2e")
  for et in ("vsd", "mssd"):
    p = ece.parse_args(["--error_type", et, "--n_top", "-1", "--datasets_path",
                        os.path.join(e2e, "datasets")])
    dp_split = dataset_params.get_split_params(p["datasets_path"], "lmo", "test")
    dp_model = dataset_params.get_model_params(p["datasets_path"], "lmo", "eval")
    targets = inout.load_json(os.path.join(dp_split["base_path"], p["targets_filename"]))
    ests = inout.load_bop_results(os.path.join(e2e, "results", "synth_lmo-test.csv"))
    t_org, e_org = ece.organize(targets, ests)
    info = inout.load_json(dp_model["models_info_path"], keys_to_int=True)
    scene_gt = inout.load_scene_gt(dp_split["scene_gt_tpath"].format(scene_id=2))
    cams = inout.load_scene_camera(dp_split["scene_camera_tpath"].format(scene_id=2))
    recs, _ = ece.scene_records(p, 2, t_org[2], e_org, scene_gt)
    ev = _FakeEv(info)
    errs, todo = ece.plan(p, recs, info)
    c = ece.todo_costs(ev.objects, p, recs, todo, cams, dp_split["im_size"])
    assert c.shape == (len(todo),) and (c > 0).all()
    if et == "mssd":
      o = [ev.objects[recs[ri]["obj_id"]] for ri, _, _, _ in todo]
      assert np.allclose(c, [x["nv"] * (18 + 28 * x["ns"]) for x in o])
    else:
      assert np.ptp(c) > 0
    parts = ece.shard_todo(recs, todo, 3, c)
    assert np.array_equal(np.sort(np.concatenate(parts)), np.arange(len(todo)))


def _multi_meta():
  from bop_toolkit_amd import synth
  meta = []
  for o in range(30):
    pts, faces = synth.superellipsoid(8, 12, (30.0 + o, 40.0, 50.0 - o), 0.7)
    meta.append({"nv": len(pts), "nf": len(faces), "ns": 1 + o % 8,
                 "bbox": (pts.min(0), pts.max(0))})
  return meta


def _multi_worker(rank, world, port, out_path):
  import bench
  from bop_toolkit_amd import synth
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  pl = bench.plan_multi(bench.CONFIGS[5], _multi_meta(), 3000, 7, rank, world, synth.TLESS_K,
                        720, 540)
  n = len(pl["gid"])
  assert pl["counts"][rank] == n
  # rows: a function of the tuple's content (pose and object), so the gathered
  # table shows each global id got the tuple the single-rank plan has there
  rows = torch.from_numpy(np.concatenate([pl["pe"], pl["pg"], pl["obj"][:, None]], 1))
  table = shard.gather_rows(rows, torch.from_numpy(pl["gid"]), pl["n_all"], counts=pl["counts"])
  if rank == 0:
    np.save(out_path, table.numpy())
  dist.barrier()
  dist.destroy_process_group()


def test_multi_instance_plan_lpt_covers_every_tuple_once(tmp_path):
  """bench.py configs[5] under 4 ranks (gloo): images assigned by LPT on the
  §8d cost (not contiguous ranges), every tuple on exactly one rank (the
  gather checks ids are a permutation), rows equal to the one-rank plan's,
  GT instances and frames consistent with the rank's tuples, and the LPT
  loads tighter than contiguous ranges of the same images."""
  import sys
  sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
  import bench
  from bop_toolkit_amd import synth
  meta = _multi_meta()
  one = bench.plan_multi(bench.CONFIGS[5], meta, 3000, 7, 0, 1, synth.TLESS_K, 720, 540)
  assert np.array_equal(one["gid"], np.arange(one["n_all"]))
  out = str(tmp_path / "multi.npy")
  mp.spawn(_multi_worker, args=(4, _free_port(), out), nprocs=4, join=True)
  table = np.load(out)
  ref = np.concatenate([one["pe"], one["pg"], one["obj"][:, None]], 1)
  assert np.array_equal(table, ref)
  plans = [bench.plan_multi(bench.CONFIGS[5], meta, 3000, 7, r, 4, synth.TLESS_K, 720, 540)
           for r in range(4)]
  assert sorted(np.concatenate([p["gid"] for p in plans]).tolist()) == list(range(one["n_all"]))
  for p in plans:
    # every tuple's frame holds a GT instance of its object
    inst = set(zip(p["inst_f"].tolist(), p["inst_obj"].tolist()))
    assert set(zip(p["frame_idx"].tolist(), p["obj"].tolist())) <= inst
    assert p["frame_idx"].max() < p["n_img"]
  # LPT balance vs contiguous image ranges (cost = the planner's own model)
  from bop_toolkit_amd import shard
  lo = np.stack([meta[o]["bbox"][0] for o in one["obj"]])
  hi = np.stack([meta[o]["bbox"][1] for o in one["obj"]])
  roi = shard.roi_pixels(lo, hi, [one["pe"], one["pg"]], synth.TLESS_K, 720, 540)
  c = shard.tuple_cost([meta[o]["nv"] for o in one["obj"]], [meta[o]["nf"] for o in one["obj"]],
                       [meta[o]["ns"] for o in one["obj"]], roi)
  lpt = [c[p["gid"]].sum() for p in plans]
  img = one["frame_idx"]
  n_img = one["n_img"]
  contig = [c[(img >= r * n_img // 4) & (img < (r + 1) * n_img // 4)].sum() for r in range(4)]
  assert max(lpt) / np.mean(lpt) <= max(contig) / np.mean(contig) + 1e-12
  ic = shard.image_costs(img, c, n_img)
  assert max(lpt) <= np.mean(lpt) + ic.max()  # the LPT bound
