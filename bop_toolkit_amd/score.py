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
  return _scores(obj_ids, scene_ids, len(matches), tars, tps, obj_tars, obj_tps, scene_tars,
                 scene_tps, do_print)


def _scores(obj_ids, scene_ids, gt_count, tars, tps, obj_tars, obj_tps, scene_tars, scene_tps,
            do_print):
  """The scores dict of score.py:126-157 from the target / true-positive counts."""
  obj_recalls = {o: calc_recall(obj_tps[o], obj_tars[o]) for o in obj_ids}
  scene_recalls = {s: float(calc_recall(scene_tps[s], scene_tars[s])) for s in scene_ids}
  scores = {
      "recall": float(calc_recall(tps, tars)),
      "obj_recalls": obj_recalls,
      "mean_obj_recall": float(float(np.mean(list(obj_recalls.values())).squeeze())),
      "scene_recalls": scene_recalls,
      "mean_scene_recall": float(float(np.mean(list(scene_recalls.values())).squeeze())),
      "gt_count": gt_count,
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


class ArrayScorer:
  """calc_localization_scores for many match outcomes of one GT table (arrays
  in the matches file's order: scene, image, object, validity): the targets
  (valid GT instances per (object, scene, image), capped at n_top) are counted
  once; each outcome (`matched` flags) then only counts its true positives.
  The same integer counts and float expressions as calc_localization_scores,
  without building the match dicts. A valid record of an object or scene
  outside obj_ids / scene_ids raises KeyError, as the reference's lookups do."""

  def __init__(self, scene_ids, obj_ids, gt_scene, gt_im, gt_obj, gt_valid, n_top):
    self.scene_ids, self.obj_ids, self.n_top = list(scene_ids), list(obj_ids), n_top
    self.valid = np.asarray(gt_valid, bool)
    obj = np.asarray(gt_obj, np.int64)[self.valid]
    scn = np.asarray(gt_scene, np.int64)[self.valid]
    im = np.asarray(gt_im, np.int64)[self.valid]
    oix = {o: k for k, o in enumerate(self.obj_ids)}
    six = {sc: k for k, sc in enumerate(self.scene_ids)}
    for o in np.unique(obj).tolist():
      if o not in oix:
        raise KeyError(o)
    for sc in np.unique(scn).tolist():
      if sc not in six:
        raise KeyError(sc)
    lut = lambda ids, ix: np.array([ix[v] for v in ids.tolist()], np.int64) if len(ids) else \
        np.zeros(0, np.int64)
    uo, io = np.unique(obj, return_inverse=True)
    us, is_ = np.unique(scn, return_inverse=True)
    self.oi = lut(uo, oix)[io] if len(obj) else np.zeros(0, np.int64)
    self.si = lut(us, six)[is_] if len(scn) else np.zeros(0, np.int64)
    # targets: valid instances per (object, scene, image), capped at n_top
    key = (self.oi * len(self.scene_ids) + self.si) * (int(im.max()) + 1 if len(im) else 1) + \
        (im - (int(im.min()) if len(im) else 0))
    uk, first, cnt = np.unique(key, return_index=True, return_counts=True)
    if n_top > 0:
      cnt = np.minimum(n_top, cnt)
    self.obj_tars = np.bincount(self.oi[first], cnt, len(self.obj_ids)).astype(np.int64)
    self.scene_tars = np.bincount(self.si[first], cnt, len(self.scene_ids)).astype(np.int64)
    self.tars = int(cnt.sum())
    self.gt_count = len(self.valid)

  def scores(self, matched, do_print=True):
    tp = np.asarray(matched, bool)[self.valid]
    obj_tps = np.bincount(self.oi[tp], minlength=len(self.obj_ids))
    scene_tps = np.bincount(self.si[tp], minlength=len(self.scene_ids))
    return _scores(self.obj_ids, self.scene_ids, self.gt_count, self.tars, int(tp.sum()),
                   dict(zip(self.obj_ids, self.obj_tars.tolist())),
                   dict(zip(self.obj_ids, obj_tps.tolist())),
                   dict(zip(self.scene_ids, self.scene_tars.tolist())),
                   dict(zip(self.scene_ids, scene_tps.tolist())), do_print)
