#!/bin/bash
# Back-face occlusion test (BOPX_VSD_CULL=3) against mesh size: configs[3]
# workload (21 objects, YCB-V 640x480) with the superellipsoid grid scaled
# (faces = 2 * n_lat * n_lon), cull off / on, same box, REPS repetitions.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for g in "50 100" "60 125" "70 143" "80 156" "100 150"; do
    set -- $g
    for c in 0 3; do
      BOPX_VSD_CULL=$c timeout -k 10 300 python bench.py --config 3 --n-lat $1 --n-lon $2 --tuples 6252 --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/cs.json 2> gpurun_out/cs.err || { tail -30 gpurun_out/cs.err; exit 1; }
      python -c "import json,sys;d=json.load(open('gpurun_out/cs.json'));print('grid %s x %s cull %s  vsd %.3f ms'%(sys.argv[1],sys.argv[2],sys.argv[3],d['kernels']['vsd']['ms']))" $1 $2 $c
    done
  done
done
