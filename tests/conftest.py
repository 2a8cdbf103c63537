"""Shared fixtures. `-m gpu` tests need an MI355X and the built libbopx.so;
everything else runs on CPU (oracle vs golden vectors, host logic, C-ABI
exports, gloo multi-process)."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
  sys.path.insert(0, REPO)


def pytest_configure(config):
  config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libbopx.so")
  # the host-only depth decoder (g++, seconds) is built on demand, like the oracle
  io_lib = os.path.join(REPO, "bop_toolkit_amd", "lib", "libbopx_io.so")
  if not os.path.exists(io_lib):
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "bop_toolkit_amd", "csrc"),
                    "../lib/libbopx_io.so"], check=False)


@pytest.fixture(scope="session")
def golden_errors():
  return dict(np.load(os.path.join(GOLDEN, "errors.npz")))


@pytest.fixture(scope="session")
def golden_vsd():
  return dict(np.load(os.path.join(GOLDEN, "vsd.npz")))


@pytest.fixture(scope="session")
def oracle_mod():
  from oracle import oracle
  oracle.lib()
  return oracle
