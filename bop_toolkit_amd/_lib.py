"""ctypes binding of libbopx.so (the C-ABI declared in include/bopx.h).

There is no CPU fallback anywhere in bop_toolkit_amd: if the HIP library is
missing or no GPU is visible, load()/Context() raise. (The CPU restatement in
oracle/ is test infrastructure and is never imported from here.)
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BOPX_LIB", os.path.join(_HERE, "lib", "libbopx.so"))

OK, E_INVALID, E_NOT_FOUND, E_HIP, E_OOM, E_UNSUPPORTED, E_INTERNAL = 0, 1, 2, 3, 4, 5, 6
COST_STEP, COST_TLINEAR = 0, 1
VISIB_BOP18, VISIB_BOP19 = 0, 1
DELTA_F64 = 1
VSD_UNIONS = 2  # BOPX_VSD_UNIONS: union pixel counts appended to the VSD output
MAX_TAUS = 16

_d = ctypes.POINTER(ctypes.c_double)
_f = ctypes.POINTER(ctypes.c_float)
_u8 = ctypes.POINTER(ctypes.c_uint8)
_u32 = ctypes.POINTER(ctypes.c_uint32)
_i32 = ctypes.POINTER(ctypes.c_int32)
_i64 = ctypes.POINTER(ctypes.c_int64)
_I = ctypes.c_int
_I64 = ctypes.c_int64
_D = ctypes.c_double
_P = ctypes.c_void_p
_CTX = ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/bopx.h one to one.
SIGNATURES = {
    "bopx_version": (_I, []),
    "bopx_device_count": (_I, [ctypes.POINTER(_I)]),
    "bopx_create": (_I, [_I, ctypes.POINTER(_CTX)]),
    "bopx_destroy": (None, [_CTX]),
    "bopx_last_error": (ctypes.c_char_p, [_CTX]),
    "bopx_synchronize": (_I, [_CTX]),
    "bopx_stream": (_P, [_CTX]),
    "bopx_add_object": (_I, [_CTX, _I, _d, _I64, _u32, _I64]),
    "bopx_remove_object": (_I, [_CTX, _I]),
    "bopx_set_symmetries": (_I, [_CTX, _I, _d, _I64]),
    "bopx_set_symmetries_many": (_I, [_CTX, _I, _i32, _i64, _d]),
    "bopx_preload": (_I, [_CTX]),
    "bopx_object_slot": (_I, [_CTX, _I, ctypes.POINTER(_I)]),
    "bopx_mssd_batch": (_I, [_CTX, _I64, _i32, _d, _d, _d]),
    "bopx_mspd_batch": (_I, [_CTX, _I64, _i32, _d, _d, _d, _d]),
    "bopx_add_batch": (_I, [_CTX, _I64, _i32, _d, _d, _d]),
    "bopx_adi_batch": (_I, [_CTX, _I64, _i32, _d, _d, _d]),
    "bopx_proj_batch": (_I, [_CTX, _I64, _i32, _d, _d, _d, _d]),
    "bopx_vsd_batch": (_I, [_CTX, _I64, _i32, _d, _d, _i32, _f, _I64, _I, _I, _d, _D, _I, _d,
                            _I, _I, _d, _I, _d]),
    "bopx_vsd_shared_batch": (_I, [_CTX, _I64, _i32, _d, _i32, _I64, _i32, _i32, _f, _I64, _I,
                                   _I, _d, _D, _I, _d, _I, _I, _d, _I, _d]),
    "bopx_vsd_shared_batch_dev": (_I, [_CTX, _I64, _P, _P, _P, _I64, _P, _P, _P, _I, _I, _P, _D,
                                       _I, _d, _I, _I, _P, _I, _P, _P]),
    "bopx_vsd_from_depths": (_I, [_CTX, _I, _I, _f, _f, _f, _D, _D, _D, _D, _D, _I, _d, _I, _I,
                                  _D, _I, _d]),
    "bopx_cover_batch": (_I, [_CTX, _I64, _i32, _d, _d, _i32, _I64, _I, _I, _d, _d]),
    "bopx_cover_from_depths": (_I, [_CTX, _I, _I, _f, _f, _d]),
    "bopx_cover_batch_dev": (_I, [_CTX, _I64, _P, _P, _P, _P, _I, _I, _P, _P, _P]),
    "bopx_gt_info_batch": (_I, [_CTX, _I64, _i32, _d, _i32, _f, _I64, _I, _I, _d, _D, _I, _I,
                                _d, _u8]),
    "bopx_gt_info_batch_dev": (_I, [_CTX, _I64, _P, _P, _P, _P, _I, _I, _P, _D, _I, _I, _P, _P,
                                    _P]),
    "bopx_render_depth": (_I, [_CTX, _I, _d, _d, _D, _D, _D, _D, _I, _I, _f]),
    "bopx_dist_im": (_I, [_CTX, _I, _I, _f, _D, _D, _D, _D, _d]),
    "bopx_visib_mask": (_I, [_CTX, _I64, _d, _d, _u8, _D, _I, _I, _u8]),
    "bopx_mssd_batch_dev": (_I, [_CTX, _I64, _P, _P, _P, _P, _P]),
    "bopx_mspd_batch_dev": (_I, [_CTX, _I64, _P, _P, _P, _P, _P, _P]),
    "bopx_add_batch_dev": (_I, [_CTX, _I64, _P, _P, _P, _P, _P]),
    "bopx_adi_batch_dev": (_I, [_CTX, _I64, _P, _P, _P, _P, _P]),
    "bopx_proj_batch_dev": (_I, [_CTX, _I64, _P, _P, _P, _P, _P, _P]),
    "bopx_vsd_batch_dev": (_I, [_CTX, _I64, _P, _P, _P, _P, _P, _I, _I, _P, _D, _I, _d, _I, _I,
                                _P, _I, _P, _P]),
    "bopx_depth_clear_dev": (_I, [_CTX, _P, _I64, _P]),
    "bopx_render_depth_batch_dev": (_I, [_CTX, _I64, _P, _P, _P, _P, _P, _I, _I, _P]),
    "bopx_depth_finish_dev": (_I, [_CTX, _P, _I64, _P]),
    "bopx_png_decode_dev": (_I, [_CTX, _I64, _P, _P, _P, _I, _I, _P, _P, _I64, _P, _P, _P]),
}

_lib = None
_lock = threading.Lock()


class BopxError(RuntimeError):
  pass


class BopxOOMError(BopxError):
  """BOPX_E_OOM: device scratch did not fit (the caller may split the batch or
  take a path with a smaller footprint)."""


def load():
  """Load libbopx.so (raises ImportError if it has not been built)."""
  global _lib
  with _lock:
    if _lib is None:
      # One HIP runtime per process: torch ships its own libamdhip64 (SONAME
      # libamdhip64.so.7, like /opt/rocm's). Loading torch first lets the
      # dynamic linker bind libbopx's NEEDED libamdhip64.so.7 to torch's copy;
      # the other order leaves two runtimes and torch then finds no GPU.
      try:
        import torch  # noqa: F401
      except ImportError:
        pass
      if not os.path.exists(LIB_PATH):
        raise ImportError(
            "libbopx.so not found at %s: build it with `python -c 'import __graft_entry__ as g;"
            " g.build()'` (bop_toolkit_amd has no CPU fallback)" % LIB_PATH)
      L = ctypes.CDLL(LIB_PATH)
      for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
      _lib = L
  return _lib


def ptr(a, ct):
  return a.ctypes.data_as(ct) if a is not None else None


def cast_ptr(addr, ct):
  """Pointer of type ct at a raw address (an offset into an array whose
  lifetime the caller holds)."""
  return ctypes.cast(addr, ct)


def device_count():
  n = _I(0)
  load().bopx_device_count(ctypes.byref(n))
  return n.value


class Context:
  """One libbopx context (a HIP device + stream + the resident object registry)."""

  def __init__(self, device=0):
    L = load()
    h = _CTX()
    rc = L.bopx_create(int(device), ctypes.byref(h))
    if rc != OK or not h.value:
      raise BopxError("bopx_create(device=%d) failed (rc=%d): no usable HIP device; "
                      "bop_toolkit_amd has no CPU fallback" % (device, rc))
    self.h = h
    self.device = int(device)
    self.lib = L

  def close(self):
    if self.h is not None and self.h.value:
      self.lib.bopx_destroy(self.h)
    self.h = None

  def __del__(self):
    try:
      self.close()
    except Exception:
      pass

  def check(self, rc, what=""):
    if rc == OK:
      return
    msg = self.lib.bopx_last_error(self.h).decode(errors="replace")
    if rc == E_INVALID:
      raise ValueError(msg)
    if rc == E_NOT_FOUND:
      raise KeyError(msg)
    if rc == E_OOM:
      raise BopxOOMError("%s failed (rc=%d): %s" % (what, rc, msg))
    raise BopxError("%s failed (rc=%d): %s" % (what, rc, msg))

  def call(self, name, *args):
    self.check(getattr(self.lib, name)(self.h, *args), name)

  def stream(self):
    return self.lib.bopx_stream(self.h)

  def slot(self, obj_id):
    s = _I(-1)
    rc = self.lib.bopx_object_slot(self.h, int(obj_id), ctypes.byref(s))
    if rc != OK:
      raise KeyError("unknown obj_id %r" % (obj_id,))
    return s.value

  # -- registry ---------------------------------------------------------------
  def add_object(self, obj_id, pts, faces=None):
    pts = np.ascontiguousarray(pts, np.float64).reshape(-1, 3)
    if faces is None:
      faces = np.zeros((0, 3), np.uint32)
    faces = np.ascontiguousarray(faces, np.uint32).reshape(-1, 3)
    self.call("bopx_add_object", int(obj_id), ptr(pts, _d), len(pts), ptr(faces, _u32),
              len(faces))

  def remove_object(self, obj_id):
    self.call("bopx_remove_object", int(obj_id))

  def set_symmetries(self, obj_id, syms12):
    syms12 = np.ascontiguousarray(syms12, np.float64).reshape(-1, 12)
    self.call("bopx_set_symmetries", int(obj_id), ptr(syms12, _d), len(syms12))

  def preload(self):
    """bopx_preload: the GPU code objects loaded now (returns the status;
    touches no other context state, so it may run on a thread of its own)."""
    return self.lib.bopx_preload(self.h)

  def set_symmetries_many(self, obj_ids, syms12_list):
    ids = np.ascontiguousarray(obj_ids, np.int32)
    arrs = [np.asarray(x, np.float64).reshape(-1, 12) for x in syms12_list]
    ns = np.array([len(x) for x in arrs], np.int64)
    rows = np.ascontiguousarray(np.concatenate(arrs) if arrs else np.zeros((0, 12)))
    self.call("bopx_set_symmetries_many", len(ids), ptr(ids, _i32), ptr(ns, _i64),
              ptr(rows, _d))


def code_object_digests(path=None):
  """sha256 of each gfx950 code object in libbopx.so's .hip_fatbin section,
  keyed by the kernels it defines ("k_vsd", "k_sym_error", "k_png_inflate",
  ...: each translation unit's kernels share one code object). Ties a
  rocprofv3 PMC summary to the machine code it measured, independently of
  host code or other translation units linked into the same library
  (bench.py load_traffic, tools/pmc.sh). Reads the file only (no GPU)."""
  import hashlib
  import re
  import struct
  with open(path or LIB_PATH, "rb") as f:
    so = f.read()
  # ELF64 section headers: find .hip_fatbin
  shoff, = struct.unpack_from("<Q", so, 0x28)
  shentsize, shnum, shstrndx = struct.unpack_from("<HHH", so, 0x3A)
  sec = [struct.unpack_from("<IIQQQQ", so, shoff + i * shentsize) for i in range(shnum)]
  stroff = sec[shstrndx][4]
  fat = None
  for name, _typ, _flags, _addr, off, size in sec:
    end = so.index(b"\0", stroff + name)
    if so[stroff + name:end] == b".hip_fatbin":
      fat = so[off:off + size]
  if fat is None:
    raise ValueError("%s has no .hip_fatbin section" % (path or LIB_PATH))
  magic = b"__CLANG_OFFLOAD_BUNDLE__"
  out = {}
  for m in re.finditer(re.escape(magic), fat):
    b = m.start()
    nent, = struct.unpack_from("<Q", fat, b + len(magic))
    p = b + len(magic) + 8
    for _ in range(nent):
      off, size, tlen = struct.unpack_from("<QQQ", fat, p)
      triple = fat[p + 24:p + 24 + tlen].decode(errors="replace")
      p += 24 + tlen
      if "gfx950" not in triple or size == 0:
        continue
      co = fat[b + off:b + off + size]
      digest = hashlib.sha256(co).hexdigest()
      # kernel descriptors are named "<mangled kernel>.kd" in the symbol table
      for k in set(re.findall(rb"(k_[a-z0-9_]+)[A-Za-z0-9_]*\.kd\0", co)):
        out[k.decode()] = digest
  return out
