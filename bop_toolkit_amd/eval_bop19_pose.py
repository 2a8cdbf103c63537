"""Counterpart of scripts/eval_bop19_pose.py: the BOP19 evaluation of result
files — VSD, MSSD, MSPD errors, recall at every threshold, average recalls.

Same parameters, command line and output files (per-error errors_*.json,
matches_*/scores_* per threshold, scores_bop19.json; eval_bop19_pose.py:17-258).
The reference spawns one interpreter per error type and one per (tau,
threshold) pair for the scores (130 processes per result file); here both
steps run in-process with the same argument strings: the error types as GPU
batches (eval_calc_errors.run), the 120 score settings against one cache of
the dataset files (eval_calc_scores.score_error_dir).
"""
import argparse
import copy
import os
import time

import numpy as np

from . import eval_calc_errors as ece
from . import eval_calc_scores as ecs
from . import inout, misc

_TH = np.arange(0.05, 0.51, 0.05)
DEFAULTS = {
    "errors": [
        {"n_top": -1, "type": "vsd",
         "vsd_deltas": {"hb": 15, "icbin": 15, "icmi": 15, "itodd": 5, "lm": 15, "lmo": 15,
                        "ruapc": 15, "tless": 15, "tudl": 15, "tyol": 15, "ycbv": 15,
                        "hope": 15},
         "vsd_taus": list(_TH), "vsd_normalized_by_diameter": True,
         "correct_th": [[th] for th in _TH]},
        {"n_top": -1, "type": "mssd", "correct_th": [[th] for th in _TH]},
        {"n_top": -1, "type": "mspd", "correct_th": [[th] for th in np.arange(5, 51, 5)]},
    ],
    "visib_gt_min": -1,
    "max_sym_disc_step": 0.01,
    "renderer_type": "vispy",
    "result_filenames": ["/relative/path/to/csv/with/results"],
    "results_path": "/path/to/results",
    "eval_path": "/path/to/eval/folder",
    "targets_filename": "test_targets_bop19.json",
}


def parse_args(argv=None):
  p = copy.deepcopy(DEFAULTS)
  ap = argparse.ArgumentParser()
  for k in ("renderer_type", "results_path", "eval_path", "targets_filename"):
    ap.add_argument("--" + k, default=p[k])
  ap.add_argument("--result_filenames", default=",".join(p["result_filenames"]))
  a = ap.parse_args(argv)
  for k in ("renderer_type", "results_path", "eval_path", "targets_filename"):
    p[k] = str(getattr(a, k))
  p["result_filenames"] = a.result_filenames.split(",")
  return p


def average_time_per_image(ests):
  """Mean of the per-image times; -1 when any is missing (negative); a
  ValueError if estimates of one image disagree by > 1 ms (:127-149)."""
  times = {}
  for est in ests:
    key = "{:06d}_{:06d}".format(est["scene_id"], est["im_id"])
    if est["time"] < 0:
      return -1.0
    if key in times:
      if abs(times[key] - est["time"]) > 0.001:
        raise ValueError("The running time for scene {} and image {} is not the same for all "
                         "estimates.".format(est["scene_id"], est["im_id"]))
    else:
      times[key] = est["time"]
  return np.mean(list(times.values()))


def errors_argv(p, error, result_filename):
  argv = ["--n_top={}".format(error["n_top"]), "--error_type={}".format(error["type"]),
          "--result_filenames={}".format(result_filename),
          "--renderer_type={}".format(p["renderer_type"]),
          "--results_path={}".format(p["results_path"]), "--eval_path={}".format(p["eval_path"]),
          "--targets_filename={}".format(p["targets_filename"]),
          "--max_sym_disc_step={}".format(p["max_sym_disc_step"]), "--skip_missing=1"]
  if error["type"] == "vsd":
    argv += ["--vsd_deltas={}".format(",".join("{}:{}".format(k, v)
                                              for k, v in error["vsd_deltas"].items())),
             "--vsd_taus={}".format(",".join(map(str, error["vsd_taus"]))),
             "--vsd_normalized_by_diameter={}".format(error["vsd_normalized_by_diameter"])]
  return argv


def _errors_and_scores(p, result_filename, result_name, dataset, device, calc_errors, scorer,
                       owner):
  """Error files of every error type (GPU), each type's folders handed to the
  scorer as soon as they are written; the scores of every folder (rank 0),
  None elsewhere. owner receives the error type of each folder."""
  for error in p["errors"]:
    if calc_errors:
      ece.run(ece.parse_args(errors_argv(p, error, result_filename)), device)
    if scorer is None:  # scores are host bookkeeping on rank 0
      continue
    jobs = []
    if error["type"] == "vsd":
      signs = [misc.get_error_signature("vsd", error["n_top"],
                                        vsd_delta=error["vsd_deltas"][dataset], vsd_tau=tau)
               for tau in error["vsd_taus"]]
    else:
      signs = [misc.get_error_signature(error["type"], error["n_top"])]
    for sign in dict.fromkeys(signs):
      error_dir_path = os.path.join(result_name, sign)
      # the reference's command line (eval_bop19_pose.py:196-213), parsed once
      # per folder; the threshold settings differ only in correct_th[type],
      # which argparse would give as the floats of the same strings
      base = None if not error["correct_th"] else ecs.parse_args([
          "--error_dir_paths={}".format(error_dir_path),
          "--eval_path={}".format(p["eval_path"]),
          "--targets_filename={}".format(p["targets_filename"]),
          "--visib_gt_min={}".format(p["visib_gt_min"]),
          "--correct_th_{}={}".format(error["type"], ",".join(map(str, error["correct_th"][0])))])
      sps = []
      for th in error["correct_th"]:
        sp = copy.deepcopy(base)
        sp["correct_th"][error["type"]] = [float(x) for x in ",".join(map(str, th)).split(",")]
        sps.append(sp)
      jobs.append((error_dir_path, sps))
      owner.append(error["type"])
    scorer.submit(jobs)
  return scorer.results() if scorer is not None else None


def evaluate(p, device=0, calc_errors=True):
  """Evaluate every result file; returns {result_name: final_scores}.
  calc_errors=False scores errors_*.json already present under eval_path."""
  out = {}
  for result_filename in p["result_filenames"]:
    misc.log("===========")
    misc.log("EVALUATING: {}".format(result_filename))
    misc.log("===========")
    t0 = time.time()
    result_name = os.path.splitext(os.path.basename(result_filename))[0]
    dataset = str(result_name.split("_")[1].split("-")[0])
    ests = ece.cached_load(inout.load_bop_results,
                           os.path.join(p["results_path"], result_filename))
    avg_time = average_time_per_image(ests)
    owner = []
    # every (folder, threshold) setting is independent: an error type's folders
    # are scored in a process pool while the next error type runs on the GPU
    n_folders = sum(len(e["vsd_taus"]) if e["type"] == "vsd" else 1 for e in p["errors"])
    scorer = ecs.FolderScorer(n_folders) if ece._dist()[0] == 0 else None
    sym_err = [e for e in p["errors"] if e["type"] in ("mssd", "mspd")]
    if calc_errors and sym_err:
      # MSSD / MSPD symmetry sets computed on a thread during the VSD pass, for
      # the parameters that pass will parse
      from . import dataset_params
      pe = ece.parse_args(errors_argv(p, sym_err[0], result_filename))
      dp_model = dataset_params.get_model_params(pe["datasets_path"], dataset, "eval")
      if os.path.exists(dp_model["models_info_path"]):
        ece.prefetch_symmetries(dp_model["models_info_path"], pe["max_sym_disc_step"])
    try:
      folder_scores = _errors_and_scores(p, result_filename, result_name, dataset, device,
                                         calc_errors, scorer, owner)
    finally:
      if scorer is not None:
        scorer.close()
    if ece._dist()[0] != 0:
      continue
    average_recalls = {}
    for error in p["errors"]:
      recalls = [s["recall"] for o, fs in zip(owner, folder_scores) if o == error["type"]
                 for s in fs]
      average_recalls[error["type"]] = np.mean(recalls)
      misc.log("Recall scores ({}): {}".format(error["type"], " ".join(map(str, recalls))))
      misc.log("Average recall: {}".format(average_recalls[error["type"]]))
    misc.log("Evaluation of {} took {}s.".format(result_filename, time.time() - t0))
    final = {"bop19_average_recall_{}".format(e["type"]): average_recalls[e["type"]]
             for e in p["errors"]}
    final["bop19_average_recall"] = np.mean(
        [average_recalls["vsd"], average_recalls["mssd"], average_recalls["mspd"]])
    final["bop19_average_time_per_image"] = avg_time
    inout.save_json(os.path.join(p["eval_path"], result_name, "scores_bop19.json"), final)
    misc.log("FINAL SCORES:")
    for k, v in final.items():
      misc.log("- {}: {}".format(k, v))
    out[result_name] = final
  misc.log("Done.")
  return out


def main(argv=None):
  from . import shard
  _, _, local = shard.init_from_env()  # torchrun: errors sharded, scores on rank 0
  evaluate(parse_args(argv), local)


if __name__ == "__main__":
  main()
