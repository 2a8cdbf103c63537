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
STATS = {"calls": 0, "frames": 0, "pack_s": 0.0, "decode_s": 0.0, "host_s": 0.0,
         # submit's other host steps (layout stat, page-locked staging growth, waits for
         # a slot's previous upload, the launch call) and finish's wait for the kernels
         "stat_s": 0.0, "stage_s": 0.0, "slot_wait_s": 0.0, "launch_s": 0.0, "kernel_wait_s": 0.0,
         "pack_c_s": 0.0}  # the packing calls alone (host threads, GIL released)
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


def pack_threads():
  """Host threads of a packing call: BOPX_PACK_THREADS, default min(16, CPUs)."""
  v = os.environ.get("BOPX_PACK_THREADS")
  return max(1, int(v)) if v else min(16, os.cpu_count() or 1)


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
                              int(workers or pack_threads()), st.ctypes.data,
                              ctypes.byref(need))
  if rc < 0:
    raise RuntimeError("bopx_pack_depth_pngs: %d bytes needed, %d given" % (need.value, cap))
  return buf, need.value, z_off, z_len, st


class Pending:
  """A batch submitted to the device decoder (DepthDecoder.submit): frames
  being produced on the stream, the per-frame device status, and what the
  host fall-back needs."""

  def __init__(self, **kw):
    self.__dict__.update(kw)


class DepthDecoder:
  """Decodes batches of 16-bit depth PNGs of one size into device frames.

  Owns a libbopx context (one per thread, include/bopx.h; lazy=True creates
  it on first use) and two page-locked staging slots of CHUNK files each,
  reused across calls. submit() packs the files a chunk at a time on host
  threads into one slot while the other slot's bytes go up on a copy stream,
  then launches the kernels on torch's current stream (waiting for the
  copies); finish() reads the per-frame status back (the frames are final
  then) and decodes on the host what the device did not take. load() =
  finish(submit())."""

  CHUNK = 512  # files per staging slot (~0.2 GB of 640x480 depth PNGs)

  def __init__(self, device=0, lazy=False):
    self.device = int(device)
    self._ctx = None if lazy else _lib.Context(device)
    self._pinned = [None, None]
    self._copied = [None, None]  # per slot: event of its last upload
    self._copy_stream = None

  @property
  def ctx(self):
    """The libbopx context (lazy=True: created by the first decode, on the
    thread that decodes)."""
    if self._ctx is None:
      self._ctx = _lib.Context(self.device)
    return self._ctx

  def _staging(self, torch, nbytes, slot=0):
    if self._pinned[slot] is None or self._pinned[slot].numel() < nbytes:
      # grown with headroom (16 MiB steps, +50 %): chunks differ in size, and
      # each page-locked allocation costs milliseconds
      size = (max(nbytes + nbytes // 2, 1 << 24) + (1 << 24) - 1) >> 24 << 24
      self._pinned[slot] = None
      self._pinned[slot] = torch.empty(size, dtype=torch.uint8, pin_memory=True)
    return self._pinned[slot]

  def submit(self, paths, scales, H, W, torch, workers=None):
    """Pack, upload and launch (asynchronous on torch's current stream)."""
    n = len(paths)
    dev = torch.device("cuda", self.device)
    stream = torch.cuda.current_stream(dev)
    frames = torch.empty((n, H, W), dtype=torch.float32, device=dev)
    sc = np.ones(n, np.float32) if scales is None else np.asarray(
        [np.float32(float(s)) for s in scales], np.float32)
    pend = Pending(paths=paths, scales=scales, sc=sc, H=int(H), W=int(W), workers=workers,
                   frames=frames, n=n, stream=stream, host_only=n == 0 or W > MAX_WIDTH or
                   H * (2 * W + 1) > MAX_RAW, t0=time.perf_counter(), pack_s=0.0)
    if pend.host_only:  # nothing, or outside the kernel's range: host decoder in finish()
      return pend
    L = _io()
    enc = [os.fsencode(q) for q in paths]
    z_off = np.zeros(n, np.int64)
    z_len = np.zeros(n, np.int32)
    st = np.zeros(n, np.int32)
    need = ctypes.c_int64(0)
    hh = (ctypes.c_int * n)(*([int(H)] * n))
    ww = (ctypes.c_int * n)(*([int(W)] * n))
    # the whole batch's layout (file sizes, 256-byte aligned), one stat per file
    t_stat = time.perf_counter()
    L.bopx_pack_depth_pngs((ctypes.c_char_p * n)(*enc), n, hh, ww, None, 0, z_off.ctypes.data,
                           z_len.ctypes.data, 0, st.ctypes.data, ctypes.byref(need))
    _stat(stat_s=time.perf_counter() - t_stat)
    if self._copy_stream is None:
      self._copy_stream = torch.cuda.Stream(dev)
    cs = self._copy_stream
    # the compressed bytes are allocated in the copy stream's order, so the
    # uploads need not wait for the kernels already queued on `stream` (the
    # previous batch's decode): a batch is packed and uploaded while the one
    # before it decodes (z_d is recorded on `stream` below)
    with torch.cuda.stream(cs):
      z_d = torch.empty(need.value, dtype=torch.uint8, device=dev)
    nt = int(workers or pack_threads())
    for k, c0 in enumerate(range(0, n, self.CHUNK)):
      c1 = min(n, c0 + self.CHUNK)
      m = c1 - c0
      slot = k & 1
      t = time.perf_counter()
      if self._copied[slot] is not None:
        self._copied[slot].synchronize()  # the slot's previous bytes are up
      _stat(slot_wait_s=time.perf_counter() - t)
      t = time.perf_counter()
      off = np.zeros(m, np.int64)
      ln = np.zeros(m, np.int32)
      cst = np.zeros(m, np.int32)
      cneed = ctypes.c_int64(0)
      cp = (ctypes.c_char_p * m)(*enc[c0:c1])
      L.bopx_pack_depth_pngs(cp, m, hh, ww, None, 0, off.ctypes.data, ln.ctypes.data, 0,
                             cst.ctypes.data, ctypes.byref(cneed))
      t_st = time.perf_counter()
      buf = self._staging(torch, cneed.value, slot)
      t += time.perf_counter() - t_st  # (not packing)
      _stat(stage_s=time.perf_counter() - t_st)
      t_c = time.perf_counter()
      rc = L.bopx_pack_depth_pngs(cp, m, hh, ww, buf.data_ptr(), buf.numel(), off.ctypes.data,
                                  ln.ctypes.data, nt, cst.ctypes.data, ctypes.byref(cneed))
      _stat(pack_c_s=time.perf_counter() - t_c)
      if rc < 0:
        raise RuntimeError("bopx_pack_depth_pngs: %d bytes needed" % cneed.value)
      pend.pack_s += time.perf_counter() - t
      base = int(z_off[c0])
      if not np.array_equal(off + base, z_off[c0:c1]):  # a file changed size since the stat
        raise RuntimeError("depth PNG files changed while being packed")
      nbytes = int(cneed.value) - 2048  # the chunk's files (the pad is the next chunk's)
      with torch.cuda.stream(cs):
        z_d[base:base + nbytes].copy_(buf[:nbytes], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(cs)
      self._copied[slot] = ev
      z_len[c0:c1] = ln
      st[c0:c1] = cst
    stream.wait_stream(cs)  # the kernels read the uploaded bytes
    z_d.record_stream(stream)
    t1 = time.perf_counter()
    off_d = torch.from_numpy(z_off).to(dev)
    len_d = torch.from_numpy(z_len).to(dev)
    sc_d = torch.from_numpy(sc).to(dev)
    raw_stride = raw_stride_of(H, W)
    raw = torch.empty(n * raw_stride, dtype=torch.uint8, device=dev)
    status = torch.empty(2 * n, dtype=torch.int32, device=dev)
    self.ctx.call("bopx_png_decode_dev", n, z_d.data_ptr(), off_d.data_ptr(), len_d.data_ptr(),
                  int(H), int(W), sc_d.data_ptr(), raw.data_ptr(), raw_stride, frames.data_ptr(),
                  status.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
    _stat(launch_s=time.perf_counter() - t1)
    pend.__dict__.update(st=st, status=status, keep=(z_d, raw, off_d, len_d, sc_d),
                         t1=t1)
    return pend

  def finish(self, pend, torch):
    """Wait for a submitted batch: (n, H, W) float32 frames, final on return.

    May run on another thread than submit: everything here is queued on the
    batch's stream (a thread's current stream does not order after the
    batch's kernels), and the batch's stream is drained before returning."""
    frames = pend.frames
    if pend.n == 0:
      return frames
    with torch.cuda.stream(pend.stream):
      self._finish_on_stream(pend, torch)
    pend.stream.synchronize()
    return frames

  def _finish_on_stream(self, pend, torch):
    n, H, W, paths, scales, sc, workers = (pend.n, pend.H, pend.W, pend.paths, pend.scales,
                                           pend.sc, pend.workers)
    frames = pend.frames
    dev = torch.device("cuda", self.device)
    if pend.host_only:
      frames.copy_(torch.from_numpy(_host_frames(paths, scales, H, W, workers)))
      self.last_host = n
      return
    tw = time.perf_counter()
    gst = pend.status.view(n, 2)[:, 0].cpu().numpy()  # waits for the kernels
    pend.keep = None
    t2 = time.perf_counter()
    _stat(kernel_wait_s=t2 - tw)
    host = np.nonzero((pend.st != 0) | (gst != 0))[0]
    if len(host):
      arr = _host_frames([paths[k] for k in host], None if scales is None else
                         [float(sc[k]) for k in host], H, W, workers)
      frames[torch.from_numpy(host).to(dev)] = torch.from_numpy(arr).to(dev)
    self.last_host = len(host)
    _stat(calls=1, frames=n, pack_s=pend.pack_s, decode_s=t2 - pend.t0 - pend.pack_s,
          host_s=time.perf_counter() - t2)

  def load(self, paths, scales, H, W, torch, workers=None):
    """(n, H, W) float32 frames on the device: sample * (float32)scales[k]
    (scales None: 1). Raises ValueError like inout.load_depths when a file
    that the device decoder cannot take has another size."""
    return self.finish(self.submit(paths, scales, H, W, torch, workers), torch)


class GroupPrefetch:
  """Test depth of consecutive scenes decoded in shared launches, ahead of use.

  A scene's frames alone leave most of the chip idle during k_png_inflate (one
  wave per stream: a launch takes one stream's latency, ~70 ms for 640x480
  frames, whether it holds 100 or 5,000 streams; past ~3,000 frames it is
  throughput-bound, tools/png_occupancy.py). A worker thread walks the scenes
  in order, collects their PNG paths (items: (key, thunk), thunk() ->
  (paths, scales), run in the worker) until a group holds max_frames frames,
  and submits the group (DepthDecoder.submit on `stream`: chunked packing on
  host threads, uploads on a copy stream, one kernel launch), so a group's
  packing and upload overlap the previous group's kernels; a second thread
  finishes the groups in order (status readback, host fall-back) as their
  kernels end. Each scene gets its slice of its group's frames. The first
  group closes at first_frames (default max_frames). At most max_groups
  (>= 2) submitted groups wait for their consumer (device memory bound). get(key) blocks until the
  scene's frames are final and returns them (None: no images; raises the
  decoder's ValueError for a group it could not take, e.g. a frame of
  another size).
  """

  def __init__(self, device, items, H, W, torch, stream, consumer, max_frames=4096, max_groups=2,
               first_frames=None):
    import concurrent.futures as cf
    self._torch = torch
    self._items = list(items)
    self._fut = {k: cf.Future() for k, _ in self._items}
    self._left = {}  # group id -> keys not yet taken
    self._group_of = {}
    self._sem = threading.Semaphore(max(2, int(max_groups)))
    self._lock = threading.Lock()
    self._stop = False
    self.H, self.W, self.max_frames = int(H), int(W), int(max_frames)
    # the first group may be smaller (the consumer starts on it sooner)
    self.first_frames = int(max_frames if first_frames is None else max(1, first_frames))
    self.stream, self.consumer, self.device = stream, consumer, device
    self.groups = 0
    self._thread = threading.Thread(target=self._run, name="bopx-depth-groups", daemon=True)
    self._thread.start()

  def _run(self):
    # the worker's decoder (its libbopx context lives on this thread)
    self._dec = DepthDecoder(self.device, lazy=True)
    # groups are finished (status readback, host fall-back) on a thread of
    # their own, in submission order, so a group's frames are released when
    # its kernels end, not after the next group's packing
    import queue
    fin_q = queue.Queue()
    fin = threading.Thread(target=self._finisher, args=(fin_q,), name="bopx-depth-finish",
                           daemon=True)
    fin.start()
    pending, n = [], 0
    cap = self.first_frames
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
        if n >= cap:
          fin_q.put(self._submit(pending))
          pending, n, cap = [], 0, self.max_frames
      if pending and not self._stop:
        fin_q.put(self._submit(pending))
    finally:
      fin_q.put(StopIteration)
      fin.join()
      for f in self._fut.values():
        if not f.done():
          f.set_exception(RuntimeError("depth prefetch stopped"))

  def _finisher(self, q):
    while True:
      job = q.get()
      if job is StopIteration:
        return
      self._finish(job)

  def _submit(self, pending):
    torch = self._torch
    self._sem.acquire()  # at most max_groups submitted groups wait for their consumer
    if self._stop:
      return None
    gid = self.groups
    self.groups += 1
    with self._lock:
      self._left[gid] = len(pending)
      for key, _, _ in pending:
        self._group_of[key] = gid
    paths = [q for _, ps, _ in pending for q in ps]
    scales = [c for _, _, cs in pending for c in cs]
    try:
      with torch.cuda.stream(self.stream):
        pend = self._dec.submit(paths, scales, self.H, self.W, torch)
    except BaseException as e:  # noqa: BLE001
      for key, _, _ in pending:
        self._fut[key].set_exception(e)
      return None
    return pending, pend

  def _finish(self, job):
    if job is None:
      return
    pending, pend = job
    torch = self._torch
    try:
      frames = self._dec.finish(pend, torch)
      frames.record_stream(self.consumer)  # freed behind the consumer's use
    except BaseException as e:  # noqa: BLE001
      for key, _, _ in pending:
        self._fut[key].set_exception(e)
      return
    o = 0
    for key, ps, _ in pending:
      self._fut[key].set_result(frames[o:o + len(ps)])
      o += len(ps)

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
    self._thread.join(timeout=60)

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
