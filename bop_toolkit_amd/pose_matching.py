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


def match_poses(errs, error_ths, max_ests_count=0, gt_valid_mask=None):
  ths = list(error_ths)
  ranked = sorted(errs, key=lambda e: e["score"], reverse=True)
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
  by_im_obj = {}
  for e in scene_errs:
    by_im_obj.setdefault(e["im_id"], {}).setdefault(e["obj_id"], []).append(e)
  out = []
  for im_id, im_gts in scene_gt.items():
    recs = [{"scene_id": scene_id, "im_id": im_id, "obj_id": gt["obj_id"], "gt_id": gt_id,
             "est_id": -1, "score": -1, "error": -1, "error_norm": -1,
             "valid": scene_gt_valid[im_id][gt_id]} for gt_id, gt in enumerate(im_gts)]
    im_errs = by_im_obj.get(im_id, {})
    for obj_id in set(gt["obj_id"] for gt in im_gts):
      if obj_id not in im_errs:
        continue
      for m in match_poses(im_errs[obj_id], correct_th, n_top, scene_gt_valid[im_id]):
        recs[m["gt_id"]].update(est_id=m["est_id"], score=m["score"], error=m["error"],
                                error_norm=m["error_norm"])
    out += recs
  return out
