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
