"""Capture end-to-end golden outputs of the reference error-calculation script.

Runs ONLY in the build container (the read-only reference checkout is at
/root/reference). It writes a small synthetic BOP dataset in the LM-O layout
(8 objects, test scene 2, 4 images) plus a BOP19 results CSV under
tests/golden/e2e/, then runs the reference's own scripts end to end:
scripts/eval_calc_errors.py for every supported error type and n_top rule,
scripts/eval_calc_scores.py on several error folders / thresholds / GT
validity rules, and scripts/eval_bop19_pose.py (which spawns the other two
130 times). The files they write are copied to tests/golden/e2e/expected/
(errors, matches, scores) and expected_bop19/ (scores per threshold +
scores_bop19.json). They pin tuple enumeration, n_top, gates, the per-tau VSD
split, the JSON layout, error values, matching, recall and the BOP19 average
recalls of bop_toolkit_amd (tests/test_e2e_errors.py, tests/test_scores.py).
scripts/calc_gt_info.py and scripts/calc_gt_masks.py run on a copy of the
dataset; their scene_gt_info.json and masks go to expected_gt/
(tests/test_gt_side.py).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_e2e.py

Harness stubs, installed by a generated sitecustomize.py in
every reference interpreter: imageio/png are absent here, so `imageio`
is a module whose imread/imwrite are backed by Pillow and `png` an empty module;
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
import subprocess
import shutil
import sys
import tempfile

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
        ("add", -1), ("adi", -1), ("cus", -1), ("proj", -1), ("re", -1), ("te", -1),
        ("rete", -1)]


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
  cams, gts, targets, gt_info = {}, {}, [], {}
  for im in range(N_IM):
    objs = list(rng.choice(OBJ_IDS, 5, replace=False))
    objs.append(objs[0])  # two instances of one object
    # image 3: objects near and across the image border (truncated silhouettes:
    # calc_gt_info's enlarged canvas, clipped ROIs)
    xy = (420.0, 320.0) if im == 3 else (120.0, 90.0)
    Rg, tg = synth.gt_poses(rng, len(objs), z_range=(600.0, 1100.0), xy=xy)
    depth = np.zeros((H, W), np.float32)
    inst, renders = [], []
    for j, o in enumerate(objs):
      pts, faces = meshes[o]
      d = oracle.render_depth(pts, faces, Rg[j], tg[j], K[0, 0], K[1, 1], K[0, 2], K[1, 2],
                              W, H)
      renders.append(d)
      m = (d > 0) & ((depth == 0) | (d < depth))
      depth[m] = d[m]
      inst.append({"cam_R_m2c": Rg[j].reshape(-1).tolist(),
                   "cam_t_m2c": tg[j].reshape(-1).tolist(), "obj_id": int(o)})
    infos = []
    for d in renders:  # scene_gt_info.json fields used by the scores (visib_fract)
      n_all = int((d > 0).sum())
      n_vis = int(((d > 0) & (d == depth)).sum())
      infos.append({"px_count_all": n_all, "px_count_visib": n_vis,
                    "visib_fract": n_vis / n_all if n_all else 0.0})
    gt_info[str(im)] = infos
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
  with open(os.path.join(sdir, "scene_gt_info.json"), "w") as f:
    json.dump(gt_info, f, indent=1)
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
  lines.append("%d,%d,%d,0.9,%s,%s,0.5" % (  # estimate of an object with no target
      SCENE, 0, 99, " ".join(["1.0", "0.0", "0.0", "0.0", "1.0", "0.0", "0.0", "0.0", "1.0"]),
      "0.0 0.0 800.0"))
  os.makedirs(os.path.join(root, "results"))
  with open(os.path.join(root, "results", RESULT), "w") as f:
    f.write("\n".join(lines) + "\n")


# Installed in every reference interpreter (errors, scores and the BOP19 driver,
# which spawns further interpreters) through PYTHONPATH.
SITECUSTOMIZE = """
import sys, types
import numpy as np
np.float = float  # removed in NumPy 2, used by the reference's inout
from PIL import Image
imageio = types.ModuleType("imageio")
imageio.imread = lambda p: np.asarray(Image.open(p))
imageio.imwrite = lambda p, im, **kw: Image.fromarray(np.asarray(im)).save(p)
sys.modules["imageio"] = imageio
sys.modules["png"] = types.ModuleType("png")


class RendererVispy:  # fills the vispy slot of renderer.create_renderer
  def __init__(self, width, height, mode="rgb+depth", shading="phong", bg_color=None):
    self.w, self.h, self.models = width, height, {}

  def add_object(self, obj_id, model_path, **kw):
    from bop_toolkit_amd import inout
    m = inout.load_ply(model_path)
    self.models[obj_id] = (m["pts"], m["faces"])

  def render_object(self, obj_id, R, t, fx, fy, cx, cy):
    from oracle import oracle
    pts, faces = self.models[obj_id]
    return {"depth": oracle.render_depth(pts, faces, np.asarray(R, np.float64),
                                         np.asarray(t, np.float64).reshape(3), fx, fy, cx, cy,
                                         self.w, self.h)}


mod = types.ModuleType("bop_toolkit_lib.renderer_vispy")
mod.RendererVispy = RendererVispy
sys.modules["bop_toolkit_lib.renderer_vispy"] = mod

# calc_gt_info.py / calc_gt_masks.py hard-code their dataset ('gist', a local
# path) in the script body: point the split/model lookups at the golden copy.
import os as _os
if _os.environ.get("BOPX_GT_REDIRECT"):
  _path, _name, _split = _os.environ["BOPX_GT_REDIRECT"].split(":")
  from bop_toolkit_lib import dataset_params as _dp
  _gsp, _gmp = _dp.get_split_params, _dp.get_model_params
  _dp.get_split_params = lambda p, n, s, t=None: _gsp(_path, _name, _split, t)
  _dp.get_model_params = lambda p, n, t=None: _gmp(_path, _name, t)
"""

# (error folder, extra arguments) of the standalone eval_calc_scores runs
SCORE_RUNS = [
    ("error=vsd_ntop=-1_delta=15.000_tau=0.200", ["--correct_th_vsd=0.3"]),
    ("error=vsd_ntop=1_delta=15.000_tau=0.500", ["--correct_th_vsd=0.25", "--visib_gt_min=0.1"]),
    ("error=mssd_ntop=-1", ["--correct_th_mssd=0.2"]),
    ("error=mssd_ntop=0", ["--correct_th_mssd=0.35", "--visib_gt_min=0.3"]),
    ("error=mspd_ntop=-1", ["--correct_th_mspd=10"]),
    ("error=ad_ntop=-1", ["--correct_th_ad=0.1"]),
    ("error=proj_ntop=-1", ["--correct_th_proj=15"]),
    ("error=rete_ntop=-1", ["--correct_th_rete=5.0,5.0"]),
    ("error=cus_ntop=-1", ["--correct_th_cus=0.5"]),
]


def run_ref(script, args, env):
  subprocess.run([sys.executable, os.path.join(REF, "scripts", script)] + args, env=env,
                 check=True, stdout=subprocess.DEVNULL)


def gt_side(env, datasets, tmp):
  """calc_gt_info.py and calc_gt_masks.py on a copy of the dataset: scene 0 is
  a copy of scene 2 (calc_gt_masks.py processes scene_ids = [0] only) and
  models/ a copy of models_eval/ (the scripts use the default model type)."""
  import shutil as sh
  root = os.path.join(tmp, "gt")
  sh.copytree(datasets, root)
  split = os.path.join(root, "lmo", "test")
  sh.copytree(os.path.join(split, "%06d" % SCENE), os.path.join(split, "000000"))
  sh.copytree(os.path.join(root, "lmo", "models_eval"), os.path.join(root, "lmo", "models"))
  genv = dict(env, BOPX_GT_REDIRECT="%s:lmo:test" % root)
  run_ref("calc_gt_info.py", [], genv)
  run_ref("calc_gt_masks.py", [], genv)
  out = os.path.join(OUT, "expected_gt")
  os.makedirs(out)
  sh.copy(os.path.join(split, "%06d" % SCENE, "scene_gt_info.json"),
          os.path.join(out, "scene_gt_info_%06d.json" % SCENE))
  from PIL import Image
  masks = {}
  for kind in ("mask", "mask_visib"):
    d = os.path.join(split, "000000", kind)
    for fn in sorted(os.listdir(d)):
      m = np.asarray(Image.open(os.path.join(d, fn)))
      masks["%s_%s" % (kind, os.path.splitext(fn)[0])] = np.packbits(m > 0)
  np.savez_compressed(os.path.join(out, "masks_scene0.npz"), **masks)


def main():
  rng = np.random.default_rng(20250220 + 8)
  if os.path.exists(OUT):
    shutil.rmtree(OUT)
  os.makedirs(OUT)
  make_dataset(rng, OUT)
  gts = json.load(open(os.path.join(OUT, "datasets", "lmo", "test", "%06d" % SCENE,
                                    "scene_gt.json")))
  targets = json.load(open(os.path.join(OUT, "datasets", "lmo", "test_targets_bop19.json")))
  make_results(rng, OUT, gts, targets)
  datasets = os.path.join(OUT, "datasets")
  results = os.path.join(OUT, "results")
  name = os.path.splitext(RESULT)[0]
  with tempfile.TemporaryDirectory() as tmp:
    stub = os.path.join(tmp, "stub")
    os.makedirs(stub)
    with open(os.path.join(stub, "sitecustomize.py"), "w") as f:
      f.write(SITECUSTOMIZE)
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([stub, REF, REPO]),
               PYTHONDONTWRITEBYTECODE="1", BOP_PATH=datasets)
    ev = os.path.join(tmp, "eval")
    for et, n_top in RUNS:
      run_ref("eval_calc_errors.py", ["--error_type", et, "--n_top", str(n_top),
                                      "--result_filenames", RESULT, "--results_path", results,
                                      "--eval_path", ev, "--datasets_path", datasets,
                                      "--renderer_type", "vispy"], env)
    for sign, extra in SCORE_RUNS:
      run_ref("eval_calc_scores.py", ["--error_dir_paths", os.path.join(name, sign),
                                      "--eval_path", ev, "--datasets_path", datasets] + extra,
              env)
    shutil.copytree(os.path.join(ev, name), os.path.join(OUT, "expected"))
    ev19 = os.path.join(tmp, "eval19")
    run_ref("eval_bop19_pose.py", ["--result_filenames", RESULT, "--results_path", results,
                                   "--eval_path", ev19, "--renderer_type", "vispy"], env)
    keep = os.path.join(OUT, "expected_bop19")
    for root, _, files in os.walk(os.path.join(ev19, name)):
      for fn in files:
        if fn.startswith("scores_"):  # errors and matches are covered above
          dst = os.path.join(keep, os.path.relpath(os.path.join(root, fn),
                                                   os.path.join(ev19, name)))
          os.makedirs(os.path.dirname(dst), exist_ok=True)
          shutil.copy(os.path.join(root, fn), dst)
    gt_side(env, datasets, tmp)
  with open(os.path.join(OUT, "runs.json"), "w") as f:
    json.dump({"result": RESULT, "runs": RUNS, "score_runs": SCORE_RUNS,
               "depth_scale": DEPTH_SCALE}, f, indent=1)
  n = sum(len(fs) for _, _, fs in os.walk(OUT))
  print("wrote %d files under %s" % (n, OUT))


if __name__ == "__main__":
  main()
