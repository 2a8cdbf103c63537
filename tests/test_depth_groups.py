"""depth_gpu.GroupPrefetch (CPU, a stand-in decoder): scenes' frames decoded
in shared groups of about max_frames, each scene gets exactly its slice in
order, scenes without images get None, a failing group raises for its scenes
only, and at most max_groups decoded groups wait for their consumer."""
import contextlib
import threading
import time
import types

import numpy as np
import pytest

from bop_toolkit_amd import depth_gpu


class _Frames:
  def __init__(self, arr):
    self.arr = arr

  def __getitem__(self, sl):
    return _Frames(self.arr[sl])

  def __len__(self):
    return len(self.arr)

  def record_stream(self, s):
    pass


def _fake_torch():
  return types.SimpleNamespace(cuda=types.SimpleNamespace(stream=lambda s: contextlib.nullcontext()))


@pytest.fixture
def fake_decoder(monkeypatch):
  calls = []

  class Dec:
    def __init__(self, device, lazy=False):
      pass

    def submit(self, paths, scales, H, W, torch, workers=None):
      calls.append(list(paths))
      return list(paths)

    def finish(self, paths, torch):
      if any(p.startswith("bad") for p in paths):
        raise ValueError("frame of another size")
      arr = np.array([[int(p.split(":")[1])] for p in paths])  # one value per frame
      return _Frames(arr)
  monkeypatch.setattr(depth_gpu, "DepthDecoder", Dec)
  return calls


def _scene(k, n):
  return (k, lambda: (["s%d:%d" % (k, 100 * k + i) for i in range(n)], [0.1] * n))


def test_groups_and_slices(fake_decoder):
  sizes = [3, 0, 5, 2, 7, 1]
  g = depth_gpu.GroupPrefetch(0, [_scene(k, n) for k, n in enumerate(sizes)], 4, 4,
                              _fake_torch(), None, None, max_frames=6, max_groups=2)
  with g:
    for k, n in enumerate(sizes):
      f = g.get(k)
      if n == 0:
        assert f is None
      else:
        assert [int(v) for v in f.arr[:, 0]] == [100 * k + i for i in range(n)]
  # groups close once they hold >= 6 frames: [3, 5] -> 8, [2, 7] -> 9, [1]
  assert [len(c) for c in fake_decoder] == [8, 9, 1]


def test_failing_group_raises_for_its_scenes_only(fake_decoder):
  items = [_scene(0, 4), (1, lambda: (["bad:0"], [1.0])), _scene(2, 5), _scene(3, 2)]
  with depth_gpu.GroupPrefetch(0, items, 4, 4, _fake_torch(), None, None, max_frames=5) as g:
    with pytest.raises(ValueError):
      g.get(0)
    with pytest.raises(ValueError):
      g.get(1)
    assert len(g.get(2)) == 5
    assert len(g.get(3)) == 2


def test_thunk_error_reaches_the_consumer(fake_decoder):
  def boom():
    raise KeyError("scene_gt")
  with depth_gpu.GroupPrefetch(0, [_scene(0, 2), (1, boom), _scene(2, 2)], 4, 4, _fake_torch(),
                               None, None, max_frames=2) as g:
    assert len(g.get(0)) == 2
    with pytest.raises(KeyError):
      g.get(1)
    assert len(g.get(2)) == 2


def test_at_most_max_groups_wait(fake_decoder):
  items = [_scene(k, 4) for k in range(8)]
  g = depth_gpu.GroupPrefetch(0, items, 4, 4, _fake_torch(), None, None, max_frames=4,
                              max_groups=2)
  try:
    time.sleep(0.3)
    assert len(fake_decoder) == 2  # nothing taken yet: two groups submitted, the worker waits
    g.get(0)
    time.sleep(0.3)
    assert len(fake_decoder) == 3
  finally:
    g.close()
  assert not g._thread.is_alive()


def test_close_while_groups_wait(fake_decoder):
  """A consumer that stops early (an error in the scene loop): close() ends
  both threads at once, with groups packed and decoded but not taken."""
  g = depth_gpu.GroupPrefetch(0, [_scene(k, 4) for k in range(10)], 4, 4, _fake_torch(), None,
                              None, max_frames=4, max_groups=2)
  assert len(g.get(0)) == 4
  time.sleep(0.2)
  t = time.perf_counter()
  g.close()
  assert time.perf_counter() - t < 5
  assert not g._thread.is_alive()
  with pytest.raises(RuntimeError):
    g.get(9)


def test_first_group_and_release_before_next_pack(fake_decoder, monkeypatch):
  """A smaller first group (first_frames), and a group's frames are released
  as soon as it is finished, while the next group's submit (packing) is still
  running (finishing runs on its own thread)."""
  gate = threading.Event()
  sub0 = depth_gpu.DepthDecoder.submit

  def slow_submit(self, paths, scales, H, W, torch, workers=None):
    if fake_decoder:  # every group after the first waits for the gate
      gate.wait(5)
    return sub0(self, paths, scales, H, W, torch, workers)
  monkeypatch.setattr(depth_gpu.DepthDecoder, "submit", slow_submit)
  items = [_scene(k, 2) for k in range(6)]
  with depth_gpu.GroupPrefetch(0, items, 4, 4, _fake_torch(), None, None, max_frames=6,
                               first_frames=2) as g:
    t = time.perf_counter()
    assert len(g.get(0)) == 2
    assert time.perf_counter() - t < 2  # not held back by the second group's submit
    gate.set()
    for k in range(1, 6):
      assert len(g.get(k)) == 2
  assert [len(c) for c in fake_decoder] == [2, 6, 4]


def test_unused_scene_slice_ignores_the_group_error(fake_decoder):
  """a scene without VSD tuples takes its slice only so that its
  group can be freed (eval_calc_errors.release_group_slice); the group's error
  (another scene's frame of another size) must not stop the pass there, while
  the scene that uses its frames still gets it, and the group is released."""
  from bop_toolkit_amd import eval_calc_errors as ece
  items = [_scene(0, 2), (1, lambda: (["bad:0"], [1.0])), _scene(2, 4), _scene(3, 4)]
  with depth_gpu.GroupPrefetch(0, items, 4, 4, _fake_torch(), None, None, max_frames=3,
                               max_groups=2) as g:
    ece.release_group_slice(g, 0)  # no tuples in scene 0: the group's ValueError is not raised
    with pytest.raises(ValueError):
      g.get(1)  # the scene that needs the frames
    assert len(g.get(2)) == 4  # the failed group was released: later groups still come
    assert len(g.get(3)) == 4
