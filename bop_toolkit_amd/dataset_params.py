"""BOP dataset layout for the error-calculation caller (scripts/eval_calc_errors.py).

Counterpart of bop_toolkit_lib/dataset_params.py, restricted to what the
pose-error pipeline reads: object ids and the symmetric subset
(get_model_params, dataset_params.py:65-158), image size, scene ids and the
path templates of a split (get_split_params, dataset_params.py:250-638), and
the present-scene scan (:641-652). Sampling ranges (depth/azimuth/elevation)
and the training-camera files are outside the evaluated path and not kept.
"""
import glob
import os
from os.path import join

_GIST_IDS = list(range(1, 201))

# obj_ids, symmetric_obj_ids (ADI instead of ADD for 'ad'); dataset_params.py:75-124
_MODELS = {
    "lm": (list(range(1, 16)), [3, 7, 10, 11]),
    "lmo": ([1, 5, 6, 8, 9, 10, 11, 12], [10, 11]),
    "tless": (list(range(1, 31)), list(range(1, 31))),
    "tudl": (list(range(1, 4)), []),
    "tyol": (list(range(1, 22)), [3, 4, 5, 6, 7, 8, 10, 11, 12, 13, 15, 16, 17, 18, 19, 21]),
    "ruapc": (list(range(1, 15)), [8, 9, 12, 13]),
    "icmi": (list(range(1, 7)), [1, 2, 6]),
    "icbin": (list(range(1, 3)), [1]),
    "itodd": (list(range(1, 29)),
              [2, 3, 4, 5, 7, 8, 9, 11, 12, 14, 17, 18, 19, 23, 24, 25, 27, 28]),
    "hbs": ([1, 3, 4, 8, 9, 10, 12, 15, 17, 18, 19, 22, 23, 29, 32, 33], [10, 12, 18, 29]),
    "hb": (list(range(1, 34)), [6, 10, 11, 12, 13, 14, 18, 24, 29]),
    "ycbv": (list(range(1, 22)), [1, 13, 14, 16, 18, 19, 20, 21]),
    "hope": (list(range(1, 29)), None),
    "kit": (list(range(1, 122)), None),
    "bigbird": (list(range(1, 111)), None),
    "data2_real_source": (_GIST_IDS, None),
    "data2_syn_source": (_GIST_IDS, None),
    "data3_1_real_source": (_GIST_IDS, None),
    "data3_1_syn_source": (_GIST_IDS, None),
}


def get_model_params(datasets_path, dataset_name, model_type=None):
  """obj_ids, symmetric_obj_ids, model_tpath, models_info_path."""
  obj_ids, sym_ids = _MODELS[dataset_name]
  if dataset_name == "tless" and model_type is None:
    model_type = "cad"  # CAD models by default
  folder = "models" + ("_" + model_type if model_type is not None else "")
  models_path = join(datasets_path, "hb" if dataset_name == "hbs" else dataset_name, folder)
  return {"obj_ids": obj_ids, "symmetric_obj_ids": sym_ids,
          "model_tpath": join(models_path, "obj_{obj_id:06d}.ply"),
          "models_info_path": join(models_path, "models_info.json")}


def _r(a, b):
  return list(range(a, b))


def _split_spec(name, split, split_type):
  """(scene_ids, im_size, split_type, directory name) of one split."""
  if name == "lm":
    return _r(1, 16), (640, 480), split_type, name
  if name == "lmo":
    return {"train": [1, 5, 6, 8, 9, 10, 11, 12], "test": [2]}[split], (640, 480), split_type, name
  if name == "tless":
    if split == "train":
      scenes = [1] if split_type == "synthetless" else _r(1, 31)
    else:
      scenes = _r(1, 21) if split == "test" else None
    st = split_type or "primesense"
    sizes = {"train": {"primesense": (400, 400), "kinect": (400, 400), "canon": (1900, 1900),
                       "render_reconst": (1280, 1024), "pbr": (720, 540),
                       "synthetless": (400, 400)},
             "test": {"primesense": (720, 540), "kinect": (720, 540), "canon": (2560, 1920)}}
    return scenes, sizes[split][st], st, name
  if name == "tudl":
    st = "render" if (split == "train" and split_type is None) else split_type
    return _r(1, 4), (640, 480), st, name
  if name == "tyol":
    return _r(1, 22), (640, 480), split_type, name
  if name == "ruapc":
    return _r(1, 15), (640, 480), split_type, name
  if name == "icmi":
    return _r(1, 7), (640, 480), split_type, name
  if name == "icbin":
    return {"train": _r(1, 3), "test": _r(1, 4)}[split], (640, 480), split_type, name
  if name == "itodd":
    return {"train": [], "val": [1], "test": [1]}[split], (1280, 960), split_type, name
  if name in ("hbs", "hb"):
    st = split_type or "primesense"
    scenes = ({"train": [], "val": [3, 5, 13], "test": [3, 5, 13]} if name == "hbs" else
              {"train": [], "val": _r(1, 14), "test": _r(1, 14)})[split]
    return scenes, {"pbr": (640, 480), "primesense": (640, 480), "kinect": (1920, 1080)}[st], \
        st, "hb"
  if name == "ycbv":
    st = "real" if (split == "train" and split_type is None) else split_type
    if split == "train":
      scenes = {"real": _r(0, 48) + _r(60, 92), "pbr": None, "synt": _r(0, 80)}[st]
    else:
      scenes = _r(48, 60) if split == "test" else None
    return scenes, (640, 480), st, name
  if name == "hope":
    return {"train": [], "val": _r(1, 11), "test": _r(1, 41)}[split], (1920, 1080), split_type, \
        name
  if name in ("kit", "bigbird"):
    n = 121 if name == "kit" else 111
    return {"train": _r(1, n), "val": _r(1, n), "test": _r(1, n)}[split], (640, 480), \
        split_type, name
  if name in ("gist", "data2_source"):
    return {"train": _r(1, 111), "val": _r(1, 111), "test": _r(1, 111)}[split], (1920, 1080), \
        split_type, name
  raise ValueError("Unknown BOP dataset ({}).".format(name))


def get_split_params(datasets_path, dataset_name, split, split_type=None):
  """Image size, scene ids and path templates of a dataset split."""
  scenes, im_size, split_type_eff, dir_name = _split_spec(dataset_name, split, split_type)
  itodd = dataset_name == "itodd"
  rgb_ext = ".jpg" if split_type == "pbr" else ".png"
  gray_ext = ".tif" if (itodd and split_type != "pbr") else ".png"
  depth_ext = ".tif" if (itodd and split_type != "pbr") else ".png"
  split_path = join(datasets_path, dir_name, split)
  if split_type_eff is not None:
    if split_type_eff == "pbr":
      scenes = _r(0, 50)
    split_path += "_" + split_type_eff
  scene = join(split_path, "{scene_id:06d}")
  return {
      "name": dataset_name, "split": split, "split_type": split_type,
      "base_path": join(datasets_path, dataset_name),
      "depth_range": None, "azimuth_range": None, "elev_range": None,
      "im_modalities": ["gray", "depth"] if itodd else ["rgb", "depth"],
      "scene_ids": scenes, "im_size": im_size, "split_path": split_path,
      "scene_camera_tpath": join(scene, "scene_camera.json"),
      "scene_gt_tpath": join(scene, "scene_gt.json"),
      "scene_gt_info_tpath": join(scene, "scene_gt_info.json"),
      "scene_gt_coco_tpath": join(scene, "scene_gt_coco.json"),
      "gray_tpath": join(scene, "gray", "{im_id:06d}" + gray_ext),
      "rgb_tpath": join(scene, "rgb", "{im_id:06d}" + rgb_ext),
      "depth_tpath": join(scene, "depth", "{im_id:06d}" + depth_ext),
      "mask_tpath": join(scene, "mask", "{im_id:06d}_{gt_id:06d}.png"),
      "mask_visib_tpath": join(scene, "mask_visib", "{im_id:06d}_{gt_id:06d}.png"),
  }


def get_present_scene_ids(dp_split):
  """Sorted ids of the scene folders present in a split."""
  return sorted(int(os.path.basename(d)) for d in glob.glob(join(dp_split["split_path"], "*"))
                if os.path.isdir(d))
