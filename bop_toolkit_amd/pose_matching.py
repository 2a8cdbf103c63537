"""Greedy matching of pose estimates to GT poses (bop_toolkit_lib/pose_matching.py).

Host-side bookkeeping after the GPU error kernels. Same
inputs, outputs and tie behaviour as the reference:

* match_poses (pose_matching.py:9-90): estimates in order of decreasing
  score (stable), optionally only the first max_ests_count; each takes the
  not-yet-matched valid GT whose error is below the threshold in EVERY
  element and lowest-so-far in every element, scanning GT ids in the order of
  the errors dict.
* match_poses_scene (:93-160): one record per GT pose of every image, filled
  with its match (-1 fields when unmatched), estimates grouped per object.
"""


def _all_below(err, best):
  return all(err[i] < best[i] for i in range(len(best)))


def group_scene_errs(scene_errs):
  """{im_id: {obj_id: [err]}} with each list in match order (score
  descending, stable). match_poses_scene accepts it in place of the flat list,
  so the grouping and sort are done once per errors file, not per threshold."""
  by_im_obj = {}
  for e in scene_errs:
    by_im_obj.setdefault(e["im_id"], {}).setdefault(e["obj_id"], []).append(e)
  for per_obj in by_im_obj.values():
    for obj_id, lst in per_obj.items():
      if len(lst) > 1:
        per_obj[obj_id] = sorted(lst, key=lambda e: e["score"], reverse=True)
  return by_im_obj


def _match_scalar(ranked, th, max_ests_count, gt_valid_mask):
  """match_poses for one-element errors and thresholds: the same greedy
  (first GT, in errors-dict order, with the strictly lowest error < th)."""
  if max_ests_count > 0:
    ranked = ranked[:max_ests_count]
  taken = set()
  out = []
  for e in ranked:
    best_id, best, best_err = -1, th, None
    for gt_id, err in e["errors"].items():
      if gt_id in taken or (gt_valid_mask and not gt_valid_mask[gt_id]):
        continue
      if err[0] < best:
        best_id, best, best_err = gt_id, err[0], err
    if best_id >= 0:
      taken.add(best_id)
      out.append((e, best_id, best_err))
  return out


def match_poses(errs, error_ths, max_ests_count=0, gt_valid_mask=None, presorted=False):
  ths = list(error_ths)
  ranked = errs if presorted else sorted(errs, key=lambda e: e["score"], reverse=True)
  if max_ests_count > 0:
    ranked = ranked[:max_ests_count]
  taken = set()
  matches = []
  for e in ranked:
    best_id, best = -1, ths
    for gt_id, err in e["errors"].items():
      if gt_valid_mask and not gt_valid_mask[gt_id]:
        continue
      if gt_id in taken:
        continue
      if _all_below(err, best):
        best_id, best = gt_id, err
    if best_id < 0:
      continue
    taken.add(best_id)
    matches.append({"est_id": e["est_id"], "gt_id": best_id, "score": e["score"],
                    "error": best,
                    "error_norm": [best[i] / float(ths[i]) for i in range(len(ths))]})
  return matches


def match_poses_scene(scene_id, scene_gt, scene_gt_valid, scene_errs, correct_th, n_top):
  """scene_errs: the flat errors list of a scene, or group_scene_errs of it."""
  by_im_obj = scene_errs if isinstance(scene_errs, dict) else group_scene_errs(scene_errs)
  ths = list(correct_th)
  scalar = len(ths) == 1
  out = []
  for im_id, im_gts in scene_gt.items():
    valid = scene_gt_valid[im_id]
    recs = [{"scene_id": scene_id, "im_id": im_id, "obj_id": gt["obj_id"], "gt_id": gt_id,
             "est_id": -1, "score": -1, "error": -1, "error_norm": -1,
             "valid": valid[gt_id]} for gt_id, gt in enumerate(im_gts)]
    im_errs = by_im_obj.get(im_id)
    if im_errs:
      for obj_id in set(gt["obj_id"] for gt in im_gts):
        ranked = im_errs.get(obj_id)
        if ranked is None:
          continue
        if scalar and all(len(v) == 1 for e in ranked for v in e["errors"].values()):
          th = ths[0]
          for e, gt_id, err in _match_scalar(ranked, th, n_top, valid):
            recs[gt_id].update(est_id=e["est_id"], score=e["score"], error=err,
                               error_norm=[err[0] / float(th)])
          continue
        for m in match_poses(ranked, ths, n_top, valid, presorted=True):
          recs[m["gt_id"]].update(est_id=m["est_id"], score=m["score"], error=m["error"],
                                  error_norm=m["error_norm"])
    out += recs
  return out
