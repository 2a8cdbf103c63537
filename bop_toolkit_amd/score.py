"""Recall / AP scores of matched poses (bop_toolkit_lib/score.py).

Host-side: counts are integers, means use np.mean over the
same lists in the same order as the reference, so scores are identical.
"""
from collections import defaultdict

import numpy as np

from . import misc


def calc_ap(rec, pre):
  """PASCAL VOC (2010+) average precision: area under the precision envelope
  of the recall-sorted curve (score.py:12-44)."""
  order = np.argsort(rec)
  mrec = np.concatenate(([0], np.array(rec)[order], [1]))
  mpre = np.concatenate(([0], np.array(pre)[order], [0]))
  for i in range(mpre.size - 3, -1, -1):
    mpre[i] = max(mpre[i], mpre[i + 1])
  step = np.nonzero(mrec[1:] != mrec[:-1])[0] + 1
  return np.sum((mrec[step] - mrec[step - 1]) * mpre[step])


def calc_recall(tp_count, targets_count):
  return 0.0 if targets_count == 0 else tp_count / float(targets_count)


def calc_localization_scores(scene_ids, obj_ids, matches, n_top, do_print=True):
  """6D localization recall (score.py:60-157): targets = valid GT instances
  per (object, scene, image), capped at n_top per image when n_top > 0;
  true positives = valid GT poses with a matched estimate."""
  insts = {o: {s: defaultdict(int) for s in scene_ids} for o in obj_ids}
  for m in matches:
    if m["valid"]:
      insts[m["obj_id"]][m["scene_id"]][m["im_id"]] += 1
  tars = 0
  obj_tars = {o: 0 for o in obj_ids}
  scene_tars = {s: 0 for s in scene_ids}
  for o, per_scene in insts.items():
    for s, per_im in per_scene.items():
      counts = list(per_im.values())
      c = sum(np.minimum(n_top, counts)) if n_top > 0 else sum(counts)
      tars += c
      obj_tars[o] += c
      scene_tars[s] += c
  tps = 0
  obj_tps = {o: 0 for o in obj_ids}
  scene_tps = {s: 0 for s in scene_ids}
  for m in matches:
    if m["valid"] and m["est_id"] != -1:
      tps += 1
      obj_tps[m["obj_id"]] += 1
      scene_tps[m["scene_id"]] += 1
  obj_recalls = {o: calc_recall(obj_tps[o], obj_tars[o]) for o in obj_ids}
  scene_recalls = {s: float(calc_recall(scene_tps[s], scene_tars[s])) for s in scene_ids}
  scores = {
      "recall": float(calc_recall(tps, tars)),
      "obj_recalls": obj_recalls,
      "mean_obj_recall": float(float(np.mean(list(obj_recalls.values())).squeeze())),
      "scene_recalls": scene_recalls,
      "mean_scene_recall": float(float(np.mean(list(scene_recalls.values())).squeeze())),
      "gt_count": len(matches),
      "targets_count": int(tars),
      "tp_count": int(tps),
  }
  if do_print:
    misc.log("")
    misc.log("GT count:           {:d}".format(scores["gt_count"]))
    misc.log("Target count:       {:d}".format(scores["targets_count"]))
    misc.log("TP count:           {:d}".format(scores["tp_count"]))
    misc.log("Recall:             {:.4f}".format(scores["recall"]))
    misc.log("Mean object recall: {:.4f}".format(scores["mean_obj_recall"]))
    misc.log("Mean scene recall:  {:.4f}".format(scores["mean_scene_recall"]))
    misc.log("Object recalls:\n{}".format(", ".join(
        "{}: {:.3f}".format(i, v) for i, v in obj_recalls.items())))
    misc.log("Scene recalls:\n{}".format(", ".join(
        "{}: {:.3f}".format(i, v) for i, v in scene_recalls.items())))
    misc.log("")
  return scores
