#!/bin/bash
# k_vsd occlusion-test modes on large meshes: BOPX_VSD_CULL unset (automatic
# back-face test) vs 1 (far-entry region test) vs 0, configs[4] and the
# configs[3] workload with a 30k-triangle grid; same box, REPS repetitions.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for args in "--config 4" "--config 3 --n-lat 100 --n-lon 150 --tuples 6252"; do
    for c in auto 1 0; do
      envs=""; [ "$c" != auto ] && envs="BOPX_VSD_CULL=$c"
      env $envs timeout -k 10 300 python bench.py $args --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/cm.json 2> gpurun_out/cm.err || { tail -30 gpurun_out/cm.err; exit 1; }
      python -c "import json,sys;d=json.load(open('gpurun_out/cm.json'));print('%-45s cull %-4s vsd %.3f ms'%(sys.argv[1],sys.argv[2],d['kernels']['vsd']['ms']))" "$args" $c
    done
  done
done
