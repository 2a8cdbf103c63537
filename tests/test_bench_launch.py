"""bench.py's rank launcher and the PMC-summary key (CPU, no GPU).

`python bench.py --gpus N` without torchrun must start N rank processes with
the environment torch.distributed.run gives them (bench.launch_ranks), and a
PMC summary must be matched to the gfx950 code object of the kernel it
measured (bench.load_traffic via _lib.code_object_digests), not to the whole
library."""
import json
import os
import sys
import types

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def _args(gpus):
  return types.SimpleNamespace(gpus=gpus)


def test_world_of():
  assert bench.world_of(_args(1), {}) == (0, 1, 0)
  assert bench.world_of(_args(4), {}) is None  # launcher
  env = {"WORLD_SIZE": "4", "RANK": "3", "LOCAL_RANK": "3"}
  assert bench.world_of(_args(4), env) == (3, 4, 3)
  with pytest.raises(SystemExit):
    bench.world_of(_args(8), env)
  with pytest.raises(SystemExit):
    bench.world_of(_args(1), env)


def test_launch_ranks_environment(tmp_path):
  code = ("import json, os, sys; keys = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', "
          "'MASTER_PORT'); json.dump({k: os.environ[k] for k in keys}, "
          "open(os.path.join(sys.argv[1], os.environ['RANK'] + '.json'), 'w'))")
  rc = bench.launch_ranks([sys.executable, "-c", code, str(tmp_path)], 3, poll=0.02)
  assert rc == 0
  got = [json.load(open(tmp_path / ("%d.json" % r))) for r in range(3)]
  assert [g["RANK"] for g in got] == ["0", "1", "2"] == [g["LOCAL_RANK"] for g in got]
  assert {g["WORLD_SIZE"] for g in got} == {"3"}
  assert {g["MASTER_ADDR"] for g in got} == {"127.0.0.1"}
  assert len({g["MASTER_PORT"] for g in got}) == 1


def test_launch_ranks_failure_stops_the_others(tmp_path):
  # rank 1 fails at once; rank 0 would sleep for a minute and is terminated
  code = ("import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(3)\ntime.sleep(60)")
  rc = bench.launch_ranks([sys.executable, "-c", code], 2, poll=0.02)
  assert rc == 3


def test_launch_ranks_failure_is_reported(tmp_path, capfd):
  """A failing rank is named on stderr with its status."""
  code = ("import os, sys, time\nif os.environ['RANK'] == '2': sys.exit(5)\ntime.sleep(60)")
  rc = bench.launch_ranks([sys.executable, "-c", code], 3, poll=0.02)
  assert rc == 5
  err = capfd.readouterr().err
  assert "rank 2 exited with status 5; stopping the other 2 rank(s)" in err


def test_gloo_bench_flow_two_ranks_launch(tmp_path):
  """The launcher path of main(): --gpus 2 without WORLD_SIZE starts two
  processes of the same command (here with a stub for the rank body)."""
  stub = tmp_path / "stub.py"
  stub.write_text(
      "import os, sys\nsys.path.insert(0, %r)\nimport bench\n"
      "a = type('A', (), {'gpus': 2})()\nrw = bench.world_of(a)\n"
      "if rw is None:\n  sys.exit(bench.launch_ranks([sys.executable, __file__], 2, poll=0.02))\n"
      "open(os.path.join(%r, 'r%%d_of_%%d' %% (rw[0], rw[1])), 'w').close()\n"
      % (REPO, str(tmp_path)))
  env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
  import subprocess
  r = subprocess.run([sys.executable, str(stub)], env=env, timeout=120)
  assert r.returncode == 0
  assert (tmp_path / "r0_of_2").exists() and (tmp_path / "r1_of_2").exists()


def test_code_object_digests_name_the_measured_kernels():
  from bop_toolkit_amd import _lib
  if not os.path.exists(_lib.LIB_PATH):
    pytest.skip("libbopx.so not built")
  d = _lib.code_object_digests()
  for k in ("k_vsd", "k_vsd_pair", "k_sym_error", "k_mean_error", "k_adi", "k_png_inflate"):
    assert len(d.get(k, "")) == 64, k
  assert d["k_vsd"] == d["k_vsd_pair"]          # one translation unit: kern_vsd.hip
  assert d["k_sym_error"] == d["k_adi"]         # kern_pose.hip
  assert len({d["k_vsd"], d["k_sym_error"], d["k_png_inflate"]}) == 3


def test_load_traffic_keyed_on_code_object(tmp_path, monkeypatch):
  """A PMC summary counts when its k_vsd code object and workload match,
  whatever the rest of the library; a different code object does not."""
  from bop_toolkit_amd import _lib
  if not os.path.exists(_lib.LIB_PATH):
    pytest.skip("libbopx.so not built")
  args = types.SimpleNamespace(config=3, objects=21, n_lat=50, n_lon=100, axes_scale=1.0, seed=5)
  key = bench.workload_key(args, 1000)
  code = bench.code_digests()
  prof = tmp_path / "profiles"
  prof.mkdir()
  monkeypatch.setattr(bench, "REPO", str(tmp_path))
  summ = {"k_vsd": {"hbm_bytes_per_launch": 123.0},
          "_meta": {"lib_sha256": "0" * 64, "code_sha256": code, "workload": key}}
  (prof / "x_pmc.json").write_text(json.dumps(summ))
  assert bench.load_traffic("vsd", args, 1000) == 123.0
  assert bench.load_traffic("vsd", args, 999) is None  # another workload
  summ["_meta"]["code_sha256"] = dict(code, k_vsd="f" * 64)
  (prof / "x_pmc.json").write_text(json.dumps(summ))
  assert bench.load_traffic("vsd", args, 1000) is None


def test_committed_pmc_matches_the_shipped_kernels(monkeypatch):
  """The driver's bench line carries `roofline.traffic` only if a committed
  PMC summary records this build's k_vsd code object and the default
  workload: after a kernel change the PMC passes must be collected again
  (tools/pmc.sh)."""
  from bop_toolkit_amd import _lib
  if not os.path.exists(_lib.LIB_PATH):
    pytest.skip("libbopx.so not built")
  monkeypatch.setattr(sys, "argv", ["bench.py"])
  args = bench.parse()
  n = (args.tuples + 5) // 6 * 6  # build_workload: whole images of 6 objects
  assert bench.load_traffic("vsd", args, n) is not None
  assert bench.load_traffic("mssd", args, n) is not None


def test_parity_max_diff():
  """bench._max_diff (the parity leg's point-error check): infinities must
  coincide in place and sign, finite values compare by max abs / rel."""
  import numpy as np
  inf = float("inf")
  assert bench._max_diff([1.0, inf], [1.0, inf]) == (0.0, 0.0)
  assert bench._max_diff([1.0, inf], [1.0, 2.0]) == (inf, inf)
  assert bench._max_diff([inf], [-inf]) == (inf, inf)
  assert bench._max_diff([inf, inf], [inf, inf]) == (0.0, 0.0)
  a, r = bench._max_diff(np.array([2.0, 4.0 + 1e-6]), np.array([2.0, 4.0]))
  assert abs(a - 1e-6) < 1e-12 and abs(r - 2.5e-7) < 1e-12
  assert set(bench.PARITY_TUPLES) == {0, 1, 2, 3, 4, 5}
  assert all(c in bench.CONFIGS for c in bench.PARITY_TUPLES)


def test_parity_leg_survives_a_failing_configuration(monkeypatch):
  """A configuration whose parity run raises is reported in its row and turns
  all_ok off; the other configurations still run and the line still prints."""
  import torch
  calls = []

  def fake(c, args, torch_, oracle, synth, ev_cls, res, png_src):
    calls.append(c)
    if c == 2:
      raise RuntimeError("boom")
    res[str(c)] = {"tuples": 1}
    return True
  monkeypatch.setattr(bench, "parity_config", fake)
  monkeypatch.setattr(torch.cuda, "empty_cache", lambda: None)
  out = bench.parity_leg(object(), torch, skip=(3,))
  assert calls == [0, 1, 2, 4, 5]
  assert out["all_ok"] is False and "boom" in out["configs"]["2"]["error"]
  assert out["configs"]["4"] == {"tuples": 1} and out["png"] is None
