#!/bin/bash
# Tile-parallel mode crossover at mid-size batches: S = 1, 2, 4 at 384..4096 tuples.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/split_big.jsonl
for s in 1 2 4; do
  BOPX_VSD_SPLIT=$s timeout -k 10 200 python tools/split_sweep.py 384,512,768,1024,1536,2048,4096 >> gpurun_out/split_big.jsonl 2> gpurun_out/split_big.err || { tail -20 gpurun_out/split_big.err; exit 1; }
  tail -1 gpurun_out/split_big.jsonl
done
