"""Test depth decoded on the GPU: the device side of inout.load_depths.

The reference reads every test depth image with inout.load_depth
(bop_toolkit_lib/inout.py:39-46, imageio) and scales it in float32
(scripts/eval_calc_errors.py:242-243, calc_gt_info.py:106-107). On the host
that is ~4 ms per 640x480 frame and core, most of it zlib inflate. Here the
host only reads the files and checks their chunks (libbopx_io.so
bopx_pack_depth_pngs: signature, CRCs, IHDR), concatenating the IDAT payloads
of a whole batch into one page-locked buffer; one DMA moves the compressed
bytes, and kern_png.hip inflates, unfilters and scales them straight into the
(n, H, W) float32 frames the VSD kernels read (bopx_png_decode_dev).

Exactness: PNG is lossless and both decoders compute sample * (float)scale in
float32, so the frames are bit-identical to the host decoder's
(tests/test_gpu_png.py). Files the device decoder does not take — another
format or size, or any defect it detects (it accepts only what the host's
libdeflate accepts, with the same bytes) — are decoded by inout.load_depths on
the host, which gives the host path's own result or raises its own error.
"""
import ctypes
import os
import threading
import time

import numpy as np

from . import _lib, inout

RAW_ALIGN = 1024      # bopx_png_decode_dev's raw_stride granule
MAX_WIDTH = 4096      # kern_png.hip's carry row (bopx_internal.h kPngMaxWidth)
MAX_RAW = 1 << 28     # inflated bytes per frame (bopx_internal.h kPngMaxRaw)


# Cumulative wall time of DepthDecoder.load's steps over all decoders
# (diagnostics for tools/e2e_bench.py): pack = reading and checking the files
# on host threads; decode = upload + kernels + status readback; host = frames
# the device did not take.
STATS = {"calls": 0, "frames": 0, "pack_s": 0.0, "decode_s": 0.0, "host_s": 0.0}
_STATS_LOCK = threading.Lock()


def _stat(**kw):
  with _STATS_LOCK:
    for k, v in kw.items():
      STATS[k] += v


def enabled():
  """BOPX_DEPTH_GPU=0 keeps the test depth on the host decoder."""
  return os.environ.get("BOPX_DEPTH_GPU", "1") != "0"


def _io():
  L = inout._io_lib()
  if not getattr(L, "_pack_sig", False):
    L.bopx_pack_depth_pngs.argtypes = [
        ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.POINTER(ctypes.c_int),
        ctypes.POINTER(ctypes.c_int), ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
    L.bopx_pack_depth_pngs.restype = ctypes.c_int
    L._pack_sig = True
  return L


def pack(paths, H, W, buf_for, workers=None):
  """Read and pack the files (bopx_pack_depth_pngs). buf_for(nbytes) returns
  a writable uint8 buffer (numpy array or a page-locked torch tensor) of at
  least nbytes. Returns (buf, need, z_off, z_len, status)."""
  n = len(paths)
  L = _io()
  cp = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
  hh = (ctypes.c_int * n)(*([int(H)] * n))
  ww = (ctypes.c_int * n)(*([int(W)] * n))
  z_off = np.zeros(n, np.int64)
  z_len = np.zeros(n, np.int32)
  st = np.zeros(n, np.int32)
  need = ctypes.c_int64(0)
  L.bopx_pack_depth_pngs(cp, n, hh, ww, None, 0, z_off.ctypes.data, z_len.ctypes.data, 0,
                         st.ctypes.data, ctypes.byref(need))
  buf = buf_for(need.value)
  addr = buf.ctypes.data if isinstance(buf, np.ndarray) else buf.data_ptr()
  cap = buf.nbytes if isinstance(buf, np.ndarray) else buf.numel() * buf.element_size()
  rc = L.bopx_pack_depth_pngs(cp, n, hh, ww, addr, cap, z_off.ctypes.data, z_len.ctypes.data,
                              int(workers or min(16, os.cpu_count() or 1)), st.ctypes.data,
                              ctypes.byref(need))
  if rc < 0:
    raise RuntimeError("bopx_pack_depth_pngs: %d bytes needed, %d given" % (need.value, cap))
  return buf, need.value, z_off, z_len, st


class Packed:
  """A batch packed for the device decoder (DepthDecoder.pack): the staging
  buffer holding the concatenated IDAT payloads and the per-file offsets,
  lengths and host-side status."""

  def __init__(self, **kw):
    self.__dict__.update(kw)


class DepthDecoder:
  """Decodes batches of 16-bit depth PNGs of one size into device frames.

  Owns a libbopx context (one per thread, include/bopx.h) and page-locked
  staging buffers reused across calls (`slot` 0 / 1: a batch can be packed
  into one while the other's upload is in flight). load() = decode(pack()):
  enqueues on torch's current stream of the device and returns once the
  frames are final (it reads the per-frame status back)."""

  def __init__(self, device=0, lazy=False):
    self.device = int(device)
    self._ctx = None if lazy else _lib.Context(device)
    self._pinned = [None, None]

  @property
  def ctx(self):
    """The libbopx context (lazy=True: created by the first decode, on the
    thread that decodes)."""
    if self._ctx is None:
      self._ctx = _lib.Context(self.device)
    return self._ctx

  def _staging(self, torch, nbytes, slot=0):
    if self._pinned[slot] is None or self._pinned[slot].numel() < nbytes:
      self._pinned[slot] = None
      self._pinned[slot] = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, pin_memory=True)
    return self._pinned[slot]

  def pack(self, paths, scales, H, W, torch, workers=None, slot=0):
    """Host half of load(): read and check the files into staging slot `slot`
    (no GPU work; the slot must not be in use by an unfinished decode)."""
    n = len(paths)
    sc = np.ones(n, np.float32) if scales is None else np.asarray(
        [np.float32(float(s)) for s in scales], np.float32)
    t0 = time.perf_counter()
    host_only = n == 0 or W > MAX_WIDTH or H * (2 * W + 1) > MAX_RAW  # outside the kernel's range
    buf = need = z_off = z_len = st = None
    if not host_only:
      buf, need, z_off, z_len, st = pack(paths, H, W, lambda nb: self._staging(torch, nb, slot),
                                         workers)
    return Packed(paths=paths, scales=scales, sc=sc, H=int(H), W=int(W), workers=workers,
                  host_only=host_only, buf=buf, need=need, z_off=z_off, z_len=z_len, st=st,
                  pack_s=time.perf_counter() - t0)

  def decode(self, pk, torch):
    """Device half of load(): upload, kernels, status, host fall-back for the
    frames the device did not take. Returns the (n, H, W) float32 frames."""
    n, H, W, paths, scales, sc, workers = (len(pk.paths), pk.H, pk.W, pk.paths, pk.scales, pk.sc,
                                           pk.workers)
    dev = torch.device("cuda", self.device)
    frames = torch.empty((n, H, W), dtype=torch.float32, device=dev)
    if n == 0:
      return frames
    if pk.host_only:
      frames.copy_(torch.from_numpy(_host_frames(paths, scales, H, W, workers)))
      torch.cuda.current_stream(dev).synchronize()
      self.last_host = n
      return frames
    t1 = time.perf_counter()
    stream = torch.cuda.current_stream(dev)
    z_d = pk.buf[:pk.need].to(dev, non_blocking=True)
    off_d = torch.from_numpy(pk.z_off).to(dev)
    len_d = torch.from_numpy(pk.z_len).to(dev)
    sc_d = torch.from_numpy(sc).to(dev)
    raw_stride = raw_stride_of(H, W)
    raw = torch.empty(n * raw_stride, dtype=torch.uint8, device=dev)
    status = torch.empty(2 * n, dtype=torch.int32, device=dev)
    self.ctx.call("bopx_png_decode_dev", n, z_d.data_ptr(), off_d.data_ptr(), len_d.data_ptr(),
                  int(H), int(W), sc_d.data_ptr(), raw.data_ptr(), raw_stride, frames.data_ptr(),
                  status.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
    gst = status.view(n, 2)[:, 0].cpu().numpy()  # synchronises: staging reusable after this
    del raw, z_d
    t2 = time.perf_counter()
    host = np.nonzero((pk.st != 0) | (gst != 0))[0]
    if len(host):
      arr = _host_frames([paths[k] for k in host], None if scales is None else
                         [float(sc[k]) for k in host], H, W, workers)
      frames[torch.from_numpy(host).to(dev)] = torch.from_numpy(arr).to(dev)
      # the index_put is queued on `stream`; callers consume the frames on other
      # streams (the scene prefetch threads), so the frames are final on return
      stream.synchronize()
    self.last_host = len(host)
    _stat(calls=1, frames=n, pack_s=pk.pack_s, decode_s=t2 - t1, host_s=time.perf_counter() - t2)
    return frames

  def load(self, paths, scales, H, W, torch, workers=None):
    """(n, H, W) float32 frames on the device: sample * (float32)scales[k]
    (scales None: 1). Raises ValueError like inout.load_depths when a file
    that the device decoder cannot take has another size."""
    return self.decode(self.pack(paths, scales, H, W, torch, workers), torch)


class GroupPrefetch:
  """Test depth of consecutive scenes decoded in shared launches, ahead of use.

  A scene's frames alone leave most of the chip idle during k_png_inflate (one
  wave per stream: a launch takes one stream's latency, ~70 ms for 640x480
  frames, whether it holds 100 or 5,000 streams). A packing thread walks the
  scenes in order, collects their PNG paths (items: (key, thunk), thunk() ->
  (paths, scales), run in that thread) until a group holds max_frames frames,
  and packs the group on host threads (DepthDecoder.pack) into one of two
  staging slots; a decoding thread uploads and decodes the groups in order
  (DepthDecoder.decode on `stream`), so group g + 1 is read and checked while
  group g is on the GPU. Each scene gets its slice of its group's frames. At
  most max_groups decoded groups wait for their consumer (device memory
  bound). get(key) blocks until the scene's frames are final and returns them
  (None: no images; raises the decoder's ValueError for a group it could not
  take, e.g. a frame of another size).
  """

  def __init__(self, device, items, H, W, torch, stream, consumer, max_frames=4096, max_groups=2):
    import concurrent.futures as cf
    import queue
    self._torch = torch
    self._items = list(items)
    self._fut = {k: cf.Future() for k, _ in self._items}
    self._left = {}  # group id -> keys not yet taken
    self._group_of = {}
    self._sem = threading.Semaphore(max_groups)
    self._slot_free = [threading.Semaphore(1), threading.Semaphore(1)]
    self._lock = threading.Lock()
    self._q = queue.Queue(maxsize=1)
    self._stop = False
    self.H, self.W, self.max_frames = int(H), int(W), int(max_frames)
    self.stream, self.consumer, self.device = stream, consumer, device
    self.groups = 0
    # the decoding thread creates the decoder's context (lazy); the packing
    # thread only fills its page-locked staging slots
    self._dec = DepthDecoder(device, lazy=True)
    self._packer = threading.Thread(target=self._pack_run, name="bopx-depth-pack", daemon=True)
    self._decoder = threading.Thread(target=self._decode_run, name="bopx-depth-decode",
                                     daemon=True)
    self._packer.start()
    self._decoder.start()

  def _pack_run(self):
    pending, n = [], 0
    try:
      for key, thunk in self._items:
        if self._stop:
          break
        try:
          paths, scales = thunk()
        except BaseException as e:  # noqa: BLE001 - the consumer re-raises it
          self._fut[key].set_exception(e)
          continue
        if not paths:
          self._fut[key].set_result(None)
          continue
        pending.append((key, paths, scales))
        n += len(paths)
        if n >= self.max_frames:
          self._pack(pending)
          pending, n = [], 0
      if pending and not self._stop:
        self._pack(pending)
    finally:
      self._q.put(None)  # end of groups

  def _pack(self, pending):
    gid = self.groups
    self.groups += 1
    slot = gid & 1
    self._slot_free[slot].acquire()  # the decode of group gid - 2 is done with the slot
    if self._stop:
      self._slot_free[slot].release()
      return
    paths = [q for _, ps, _ in pending for q in ps]
    scales = [c for _, _, cs in pending for c in cs]
    try:
      pk = self._dec.pack(paths, scales, self.H, self.W, self._torch, slot=slot)
    except BaseException as e:  # noqa: BLE001
      self._slot_free[slot].release()
      for key, _, _ in pending:
        self._fut[key].set_exception(e)
      return
    self._q.put((gid, slot, pending, pk))

  def _decode_run(self):
    torch = self._torch
    while True:
      job = self._q.get()
      if job is None:
        break
      gid, slot, pending, pk = job
      try:
        if not self._stop:
          self._sem.acquire()  # at most max_groups decoded groups wait for their consumer
        if self._stop:
          continue  # drain the queue (the finally frees the slot)
        with self._lock:
          self._left[gid] = len(pending)
          for key, _, _ in pending:
            self._group_of[key] = gid
        try:
          with torch.cuda.stream(self.stream):
            frames = self._dec.decode(pk, torch)
          frames.record_stream(self.consumer)  # freed behind the consumer's use
        except BaseException as e:  # noqa: BLE001
          for key, _, _ in pending:
            self._fut[key].set_exception(e)
          continue
        o = 0
        for key, ps, _ in pending:
          self._fut[key].set_result(frames[o:o + len(ps)])
          o += len(ps)
      finally:
        self._slot_free[slot].release()
    for f in self._fut.values():
      if not f.done():
        f.set_exception(RuntimeError("depth prefetch stopped"))

  def get(self, key):
    try:
      return self._fut[key].result()
    finally:
      with self._lock:
        gid = self._group_of.pop(key, None)
        if gid is not None:
          self._left[gid] -= 1
          if self._left[gid] == 0:
            del self._left[gid]
            self._sem.release()

  def close(self):
    self._stop = True
    self._sem.release()
    for sf in self._slot_free:
      sf.release()
    try:
      self._q.put_nowait(None)
    except Exception:  # noqa: BLE001 - full: the decoder still has a job; it sees _stop
      pass
    self._packer.join(timeout=60)
    self._decoder.join(timeout=60)

  def __enter__(self):
    return self

  def __exit__(self, *exc):
    self.close()
    return False


def raw_stride_of(H, W):
  """bopx_png_decode_dev's per-frame scratch: the inflated rows + 64, in KiB."""
  return (H * (2 * W + 1) + 64 + RAW_ALIGN - 1) // RAW_ALIGN * RAW_ALIGN


def _host_frames(paths, scales, H, W, workers):
  arr = np.empty((len(paths), H, W), np.float32)
  inout.load_depths(paths, scales=scales, out=arr, workers=workers)
  return arr
