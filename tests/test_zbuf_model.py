"""The raster spec returns the float32 eye Z; the reference's vispy renderer
returns its z-buffer's window depth, linearised (renderer_vispy.py:447-456,
526-536). This pins how much that difference moves VSD (DESIGN.md §4,
tools/zbuf_study.py; the 32k-tuple run is profiles/r04/zbuf_study.json):
bits 0 of the model is the spec itself, float32 and 24-bit buffers change a
fraction of a percent of the VSD rows by < 1e-3, a 16-bit buffer about half
of them by a few 1e-3, and AR_VSD moves by < 1e-5 in every case."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def sample():
  sys.path.insert(0, REPO)
  sys.path.insert(0, os.path.join(REPO, "tools"))
  import bench
  import zbuf_study as zs
  from bop_toolkit_amd import synth
  seed = 20250220 + 4
  objs = zs.bench_objects(seed)
  obj, pe, pg, _, per_img = zs.bench_poses(objs, seed, bench.CONFIGS[3]["tuples"])
  n_img = 200
  n = n_img * per_img
  K = synth.YCBV_K
  cam = (K[0, 0], K[1, 1], K[0, 2], K[1, 2])
  frames = zs.make_frames(objs, obj, pg, n_img, per_img, cam, 640, 480, seed, os.cpu_count() or 1)
  fidx = np.repeat(np.arange(n_img, dtype=np.int32), per_img)
  dia = np.array([objs[o]["diameter"] for o in obj[:n]])
  res, out = zs.study(objs, obj[:n], pe[:n], pg[:n], fidx, frames, np.tile(np.array(cam), (n_img, 1)),
                      np.arange(0.05, 0.51, 0.05), dia)
  return res, out, (objs, obj[:n], pe[:n], pg[:n], fidx, frames, np.tile(np.array(cam), (n_img, 1)),
                    dia)


def test_spec_mode_is_the_oracle_vsd(sample):
  from oracle import oracle
  res, out, (objs, obj, pe, pg, fidx, frames, cam, dia) = sample
  for o in objs:
    o.setdefault("syms", np.concatenate([np.eye(3).reshape(9), np.zeros(3)])[None])
  sel = np.arange(0, len(obj), 7)
  v, _, _ = oracle.bop19_batch(objs, obj[sel], pe[sel], pg[sel], fidx[sel], frames, cam, 15.0,
                               np.arange(0.05, 0.51, 0.05), dia[sel])
  assert np.array_equal(out[sel, 0], v)


def test_zbuffer_models_move_vsd_little(sample):
  res, out, _ = sample
  m = res["models"]
  assert res["tuples"] == 1200
  for k in ("float32", "unorm24"):
    assert m[k]["rows_changed_frac"] < 0.02, (k, m[k])
    assert max(m[k]["max_abs_dvsd_per_tau"]) < 5e-3, (k, m[k])
  assert 0.2 < m["unorm16"]["rows_changed_frac"] < 0.8, m["unorm16"]
  assert max(m["unorm16"]["max_abs_dvsd_per_tau"]) < 1e-2
  for k in m:
    assert abs(m[k]["dAR_VSD"]) < 1e-5, (k, m[k])
