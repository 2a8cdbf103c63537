"""Capture end-to-end golden outputs of the reference error-calculation script.

Runs ONLY in the build container (the read-only reference checkout is at
/root/reference). It writes a small synthetic BOP dataset in the LM-O layout
(8 objects, test scene 2, 4 images) plus a BOP19 results CSV under
tests/golden/e2e/, then runs the reference's scripts/eval_calc_errors.py
end to end with runpy for every supported error type, and copies the
errors_*.json files it writes to tests/golden/e2e/expected/. Those files
pin tuple enumeration, n_top, gates, the per-tau VSD split, the JSON layout
and the error values of bop_toolkit_amd.eval_calc_errors
(tests/test_e2e_errors.py).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_e2e.py

Harness stubs: imageio/png are absent here, so `imageio`
is a module whose imread is backed by Pillow and `png` an empty module;
NumPy 2 removed np.float, which the reference's inout uses, so it is set to
float. The reference's OpenGL renderers cannot run here: the vispy slot
(`bop_toolkit_lib.renderer_vispy`, honoured by renderer.create_renderer) is
filled by a renderer drawing with our CPU raster twin (oracle/), so the VSD
values are the reference's pipeline evaluated on depth maps that follow raster
spec v4 — the same maps k_vsd rasterises (VSD-given-depth is pinned; the
raster itself is pinned against the spec, not against OpenGL).
"""
import json
import os
import runpy
import shutil
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("BOP_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from bop_toolkit_amd import inout, synth  # noqa: E402
from oracle import oracle  # noqa: E402

OUT = os.path.join(HERE, "e2e")
W, H = 640, 480
OBJ_IDS = [1, 5, 6, 8, 9, 10, 11, 12]  # LM-O
SCENE = 2
N_IM = 4
DEPTH_SCALE = 0.1  # depth PNG in 0.1 mm units
RESULT = "synth_lmo-test.csv"
RUNS = [("vsd", -1), ("vsd", 1), ("mssd", -1), ("mssd", 0), ("mspd", -1), ("ad", -1),
        ("add", -1), ("adi", -1), ("proj", -1), ("re", -1), ("te", -1), ("rete", -1)]


def make_dataset(rng, root):
  ds = os.path.join(root, "datasets", "lmo")
  mdir = os.path.join(ds, "models_eval")
  os.makedirs(mdir)
  meshes, info = {}, {}
  for k, o in enumerate(OBJ_IDS):
    axes = tuple(rng.uniform(30.0, 80.0, 3))
    pts, faces = synth.superellipsoid(10, 40, axes, float(rng.uniform(0.5, 1.0)))
    n_disc = [1, 2, 4, 1, 8, 1, 2, 1][k]
    e = synth.models_info_entry(pts, n_disc, continuous=(o == 10))
    info[str(o)] = {kk: (float(v) if not isinstance(v, list) else v) for kk, v in e.items()}
    inout.save_ply(os.path.join(mdir, "obj_%06d.ply" % o), pts, faces)
    meshes[o] = (pts.astype(np.float64), faces)
  with open(os.path.join(mdir, "models_info.json"), "w") as f:
    json.dump(info, f, indent=1)
  sdir = os.path.join(ds, "test", "%06d" % SCENE)
  os.makedirs(os.path.join(sdir, "depth"))
  K = synth.LMO_K
  cams, gts, targets = {}, {}, []
  for im in range(N_IM):
    objs = list(rng.choice(OBJ_IDS, 5, replace=False))
    objs.append(objs[0])  # two instances of one object
    Rg, tg = synth.gt_poses(rng, len(objs), z_range=(600.0, 1100.0), xy=(120.0, 90.0))
    depth = np.zeros((H, W), np.float32)
    inst = []
    for j, o in enumerate(objs):
      pts, faces = meshes[o]
      d = oracle.render_depth(pts, faces, Rg[j], tg[j], K[0, 0], K[1, 1], K[0, 2], K[1, 2],
                              W, H)
      m = (d > 0) & ((depth == 0) | (d < depth))
      depth[m] = d[m]
      inst.append({"cam_R_m2c": Rg[j].reshape(-1).tolist(),
                   "cam_t_m2c": tg[j].reshape(-1).tolist(), "obj_id": int(o)})
    depth[depth == 0] = 1600.0
    depth[40 + 30 * im:120 + 30 * im, 200:330] = 500.0  # occluder
    depth[300:340, 100:400] = 0.0  # missing depth
    hole = rng.random((H, W)) < 0.02
    depth[hole] = 0.0
    png = np.round(depth / DEPTH_SCALE).astype(np.uint16)
    from PIL import Image
    Image.fromarray(png).save(os.path.join(sdir, "depth", "%06d.png" % im))
    cams[str(im)] = {"cam_K": K.reshape(-1).tolist(), "depth_scale": DEPTH_SCALE}
    gts[str(im)] = inst
    for o in sorted(set(objs)):
      targets.append({"im_id": im, "inst_count": int(objs.count(o)), "obj_id": int(o),
                      "scene_id": SCENE})
  with open(os.path.join(sdir, "scene_camera.json"), "w") as f:
    json.dump(cams, f, indent=1)
  with open(os.path.join(sdir, "scene_gt.json"), "w") as f:
    json.dump(gts, f, indent=1)
  with open(os.path.join(ds, "test_targets_bop19.json"), "w") as f:
    json.dump(targets, f, indent=1)
  return meshes, gts, targets


def make_results(rng, root, gts, targets):
  lines = ["scene_id,im_id,obj_id,score,R,t,time"]
  for tgt in targets:
    im, o = tgt["im_id"], tgt["obj_id"]
    gt = [g for g in gts[str(im)] if g["obj_id"] == o]
    n_est = int(rng.integers(0, 4))
    for k in range(n_est):
      g = gt[k % len(gt)]
      R = np.array(g["cam_R_m2c"]).reshape(1, 3, 3)
      t = np.array(g["cam_t_m2c"]).reshape(1, 3)
      Re, te = synth.perturb(rng, R, t, outlier_frac=0.0)
      if k == 2:
        te = te + np.array([[400.0, 0.0, 300.0]])  # far off: gated
      score = 0.5 if k == 1 else float(np.round(rng.random(), 3))  # ties possible
      lines.append("%d,%d,%d,%s,%s,%s,%s" % (
          SCENE, im, o, repr(score), " ".join(repr(float(x)) for x in Re.reshape(-1)),
          " ".join(repr(float(x)) for x in te.reshape(-1)), "0.5"))
  lines.append("%d,%d,%d,0.9,%s,%s,0.1" % (  # estimate of an object with no target
      SCENE, 0, 99, " ".join(["1.0", "0.0", "0.0", "0.0", "1.0", "0.0", "0.0", "0.0", "1.0"]),
      "0.0 0.0 800.0"))
  os.makedirs(os.path.join(root, "results"))
  with open(os.path.join(root, "results", RESULT), "w") as f:
    f.write("\n".join(lines) + "\n")


def install_stubs(meshes_by_path):
  np.float = float  # removed in NumPy 2, used by the reference's inout
  from PIL import Image
  imageio = types.ModuleType("imageio")
  imageio.imread = lambda p: np.asarray(Image.open(p))
  sys.modules["imageio"] = imageio
  sys.modules["png"] = types.ModuleType("png")
  sys.path.insert(0, REF)

  class RendererVispy:  # fills the vispy slot of renderer.create_renderer
    def __init__(self, width, height, mode="rgb+depth", shading="phong", bg_color=None):
      self.w, self.h, self.models = width, height, {}

    def add_object(self, obj_id, model_path, **kw):
      m = inout.load_ply(model_path)
      self.models[obj_id] = (m["pts"], m["faces"])

    def render_object(self, obj_id, R, t, fx, fy, cx, cy):
      pts, faces = self.models[obj_id]
      return {"depth": oracle.render_depth(pts, faces, np.asarray(R, np.float64),
                                           np.asarray(t, np.float64).reshape(3), fx, fy, cx, cy,
                                           self.w, self.h)}

  mod = types.ModuleType("bop_toolkit_lib.renderer_vispy")
  mod.RendererVispy = RendererVispy
  sys.modules["bop_toolkit_lib.renderer_vispy"] = mod
  import bop_toolkit_lib
  bop_toolkit_lib.renderer_vispy = mod


def main():
  rng = np.random.default_rng(20250220 + 8)
  if os.path.exists(OUT):
    shutil.rmtree(OUT)
  os.makedirs(OUT)
  meshes, gts, targets = make_dataset(rng, OUT)
  make_results(rng, OUT, gts, targets)
  install_stubs(meshes)
  script = os.path.join(REF, "scripts", "eval_calc_errors.py")
  expected = os.path.join(OUT, "expected")
  with tempfile.TemporaryDirectory() as ev:
    for et, n_top in RUNS:
      sys.argv = [script, "--error_type", et, "--n_top", str(n_top), "--result_filenames",
                  RESULT, "--results_path", os.path.join(OUT, "results"), "--eval_path", ev,
                  "--datasets_path", os.path.join(OUT, "datasets"), "--renderer_type", "vispy"]
      runpy.run_path(script, run_name="__main__")
    src = os.path.join(ev, os.path.splitext(RESULT)[0])
    shutil.copytree(src, expected)
  with open(os.path.join(OUT, "runs.json"), "w") as f:
    json.dump({"result": RESULT, "runs": RUNS, "depth_scale": DEPTH_SCALE}, f)
  n = sum(len(fs) for _, _, fs in os.walk(expected))
  print("wrote %d expected files under %s" % (n, expected))


if __name__ == "__main__":
  main()
