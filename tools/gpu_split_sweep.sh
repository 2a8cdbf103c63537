#!/bin/bash
# k_vsd tile-parallel mode: batch-size sweep, split off / auto / forced 4 and 16.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/split_sweep.jsonl
for s in 1 auto 4 16; do
  if [ "$s" = auto ]; then
    timeout -k 10 180 python tools/split_sweep.py >> gpurun_out/split_sweep.jsonl 2> gpurun_out/split_sweep.err || { tail -20 gpurun_out/split_sweep.err; exit 1; }
  else
    BOPX_VSD_SPLIT=$s timeout -k 10 180 python tools/split_sweep.py >> gpurun_out/split_sweep.jsonl 2> gpurun_out/split_sweep.err || { tail -20 gpurun_out/split_sweep.err; exit 1; }
  fi
  tail -1 gpurun_out/split_sweep.jsonl
done
