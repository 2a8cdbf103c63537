"""The C-ABI library loads on a CPU-only host and exports exactly the entry
points include/bopx.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "bopx.h")
LIB = os.path.join(REPO, "bop_toolkit_amd", "lib", "libbopx.so")


def declared_symbols():
  src = open(HEADER).read()
  src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
  return sorted(set(re.findall(r"\b(bopx_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_api():
  syms = declared_symbols()
  for s in ("bopx_create", "bopx_vsd_batch", "bopx_mssd_batch", "bopx_mspd_batch",
            "bopx_add_batch", "bopx_adi_batch", "bopx_render_depth", "bopx_visib_mask",
            "bopx_dist_im", "bopx_vsd_batch_dev"):
    assert s in syms


@pytest.mark.skipif(not os.path.exists(LIB), reason="libbopx.so not built")
def test_library_exports_every_declared_symbol():
  L = ctypes.CDLL(LIB)
  missing = [s for s in declared_symbols() if not hasattr(L, s)]
  assert not missing, missing


@pytest.mark.skipif(not os.path.exists(LIB), reason="libbopx.so not built")
def test_ctypes_table_matches_header():
  from bop_toolkit_amd import _lib
  assert sorted(_lib.SIGNATURES) == declared_symbols()
  L = _lib.load()
  assert L.bopx_version() >= 1


@pytest.mark.skipif(not os.path.exists(LIB), reason="libbopx.so not built")
def test_no_gpu_fails_loudly():
  """Without a GPU the product raises instead of silently falling back."""
  from bop_toolkit_amd import _lib
  if _lib.device_count() > 0:
    pytest.skip("GPU present")
  with pytest.raises(_lib.BopxError):
    _lib.Context(0)


IO_HEADER = os.path.join(REPO, "include", "bopx_io.h")
IO_LIB = os.path.join(REPO, "bop_toolkit_amd", "lib", "libbopx_io.so")


def test_io_library_exports_every_declared_symbol():
  """libbopx_io.so (host depth decoder) exports what include/bopx_io.h declares."""
  src = re.sub(r"/\*.*?\*/", "", open(IO_HEADER).read(), flags=re.S)
  syms = sorted(set(re.findall(r"\b(bopx_[a-z0-9_]+)\s*\(", src)))
  assert syms == ["bopx_decode_depth_png", "bopx_gt_lists_open", "bopx_gt_lists_take",
                  "bopx_io_backend", "bopx_load_depth_pngs", "bopx_pack_depth_pngs",
                  "bopx_read_bop_results"]
  assert os.path.exists(IO_LIB), "libbopx_io.so not built (make -C bop_toolkit_amd/csrc)"
  L = ctypes.CDLL(IO_LIB)
  assert not [s for s in syms if not hasattr(L, s)]


def test_status_codes_match_header():
  """The ctypes layer's status codes are the header's (BOPX_E_INTERNAL: a launch
  refused because the object registry's maxima are stale, runtime.cpp
  launch_dev)."""
  import re
  from bop_toolkit_amd import _lib
  hdr = open(os.path.join(REPO, "include", "bopx.h")).read()
  codes = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define BOPX_(OK|E_\w+) (\d+)", hdr)}
  for name, v in codes.items():
    assert getattr(_lib, name) == v, name
  assert codes["E_INTERNAL"] == 6
