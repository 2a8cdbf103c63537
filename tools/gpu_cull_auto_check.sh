#!/bin/bash
# The automatic back-face test (BOPX_VSD_CULL unset) against forced off (0) and
# forced on (3) on workloads either side of its mesh-size / density rule.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for args in "--config 4" "--config 3 --n-lat 100 --n-lon 150 --axes-scale 2.0 --tuples 6252" "--config 3 --n-lat 100 --n-lon 150 --axes-scale 1.5 --tuples 6252" "--config 3"; do
    for c in auto 0 3; do
      envs=""; [ "$c" != auto ] && envs="BOPX_VSD_CULL=$c"
      env $envs timeout -k 10 300 python bench.py $args --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/ca.json 2> gpurun_out/ca.err || { tail -30 gpurun_out/ca.err; exit 1; }
      python -c "import json,sys;d=json.load(open('gpurun_out/ca.json'));print('%-70s cull %-4s vsd %.3f ms'%(sys.argv[1],sys.argv[2],d['kernels']['vsd']['ms']))" "$args" $c
    done
  done
done
