"""The sharded caller path with real kernels: scripts/eval_bop19_pose.py under
torchrun with two ranks on one GPU (BOPX_DIST_BACKEND=gloo: host collectives,
the ranks share the card). Each rank evaluates its LPT share of every scene's
images; rows are gathered to rank 0, which writes the files. Every output must
be byte-identical to what the reference scripts wrote (tests/golden/e2e)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
E2E = os.path.join(REPO, "tests", "golden", "e2e")


def _free_port():
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  port = s.getsockname()[1]
  s.close()
  return port


def test_bop19_two_ranks_match_reference(tmp_path):
  import json
  runs = json.load(open(os.path.join(E2E, "runs.json")))
  name = os.path.splitext(runs["result"])[0]
  env = dict(os.environ, BOPX_DIST_BACKEND="gloo", BOP_PATH=os.path.join(E2E, "datasets"),
             BOPX_SCORE_WORKERS="2")
  cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
         "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(),
         os.path.join(REPO, "scripts", "eval_bop19_pose.py"),
         "--result_filenames", runs["result"], "--results_path", os.path.join(E2E, "results"),
         "--eval_path", str(tmp_path)]
  r = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=480)
  assert r.returncode == 0, r.stderr[-3000:]
  exp = os.path.join(E2E, "expected_bop19")
  n = 0
  for root, _, files in os.walk(exp):
    for fn in files:
      rel = os.path.relpath(os.path.join(root, fn), exp)
      with open(os.path.join(root, fn)) as f, open(tmp_path / name / rel) as g:
        assert g.read() == f.read(), rel
      n += 1
  assert n == 1 + 10 * 10 + 10 + 10
  # the VSD error files themselves (bit-identical text, like the 1-rank caller)
  for sign in os.listdir(os.path.join(E2E, "expected")):
    if not sign.startswith("error=vsd_ntop=-1"):
      continue
    with open(os.path.join(E2E, "expected", sign, "errors_000002.json")) as f, \
        open(tmp_path / name / sign / "errors_000002.json") as g:
      assert g.read() == f.read(), sign


_RCCL_GATHER = r"""
import os, torch, torch.distributed as dist
from bop_toolkit_amd import shard
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl"
g = torch.Generator().manual_seed(7)
n, c = 1000, 12
rows = torch.rand((n, c), generator=g, dtype=torch.float64).cuda()
ids = torch.randperm(n, generator=g).cuda()
for counts in (None, [n]):
  table = shard.gather_rows(rows, ids, n, counts=counts)
  ref = torch.empty_like(rows)
  ref[ids] = rows
  assert table.device.type == "cuda" and torch.equal(table, ref), counts
torch.cuda.synchronize()
dist.destroy_process_group()
print("RCCL_GATHER_OK")
"""


def test_rccl_gather_rows_one_rank():
  """shard.gather_rows over the real RCCL backend (the collective bench.py and
  the sharded callers use at N > 1: one gather of device rows to rank 0,
  scattered by tuple id there), world size 1 on this one-GPU box."""
  env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
             WORLD_SIZE="1", LOCAL_RANK="0", PYTHONPATH=REPO)
  r = subprocess.run([sys.executable, "-c", _RCCL_GATHER], env=env, cwd=REPO,
                     capture_output=True, text=True, timeout=180)
  assert r.returncode == 0 and "RCCL_GATHER_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_bench_two_ranks_strong_scaling():
  """bench.py under torchrun, 2 ranks on the one GPU (gloo host collectives):
  the job's 1,002 tuples (167 images) are split by LPT into two uneven shards,
  rows gathered to rank 0 every step; the line reports the whole job."""
  import json
  env = dict(os.environ, BOPX_DIST_BACKEND="gloo")
  cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
         "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(),
         os.path.join(REPO, "bench.py"), "--gpus", "2", "--tuples", "1000", "--steps", "2",
         "--warmup", "1", "--no-cpu-baseline"]
  r = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=300)
  assert r.returncode == 0, r.stderr[-3000:]
  line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
  assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 1002
  assert line["scaling"] == "strong" and 0 < line["config"]["tuples_rank0"] < 1002
  assert line["value"] > 0


def test_bench_two_ranks_multi_instance():
  """The multi-instance variant (shared renders) under torchrun, 2 ranks on the
  one GPU: each rank renders and evaluates its contiguous share of the images;
  the line reports the whole job."""
  import json
  env = dict(os.environ, BOPX_DIST_BACKEND="gloo")
  cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
         "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(),
         os.path.join(REPO, "bench.py"), "--gpus", "2", "--config", "5", "--tuples", "1500",
         "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
  r = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=300)
  assert r.returncode == 0, r.stderr[-3000:]
  line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
  n = line["config"]["global_batch"]
  assert line["n_gpus"] == 2 and n > 1000 and 0 < line["config"]["tuples_rank0"] < n  # ~1,500 (random k)
  assert line["value"] > 0 and line["kernels"]["vsd"]["ms"] > 0


def test_bench_gpus_flag_launches_ranks():
  """`python bench.py --gpus 2` without torchrun (the driver's command form):
  bench.py starts the two rank processes itself (gloo rehearsal on the one
  GPU), the line reports n_gpus 2 and the unchanged whole job."""
  import json
  env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
  env["BOPX_DIST_BACKEND"] = "gloo"
  cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--tuples", "1000",
         "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
  r = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=300)
  assert r.returncode == 0, r.stderr[-3000:]
  lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
  assert len(lines) == 1  # rank 0 only
  line = json.loads(lines[0])
  assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 1002
  assert 0 < line["config"]["tuples_rank0"] < 1002 and line["value"] > 0
