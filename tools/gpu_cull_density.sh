#!/bin/bash
# Does the back-face test's pay-off follow mesh size or on-screen density?
# configs[3] workload, mesh size x object size (--axes-scale), cull 0 vs 3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for g in "50 100 0.5" "50 100 0.7" "70 143 1.0" "100 150 1.5" "100 150 2.0"; do
    set -- $g
    for c in 0 3; do
      BOPX_VSD_CULL=$c timeout -k 10 300 python bench.py --config 3 --n-lat $1 --n-lon $2 --axes-scale $3 --tuples 6252 --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/cd.json 2> gpurun_out/cd.err || { tail -30 gpurun_out/cd.err; exit 1; }
      python -c "import json,sys;d=json.load(open('gpurun_out/cd.json'));print('grid %s x %s scale %s cull %s  vsd %.3f ms roi %.0f'%(sys.argv[1],sys.argv[2],sys.argv[3],sys.argv[4],d['kernels']['vsd']['ms'],d['config']['roi_mean_px']))" $1 $2 $3 $c
    done
  done
done
