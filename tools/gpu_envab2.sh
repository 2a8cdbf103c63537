#!/bin/bash
# Same-box A/B of k_vsd runtime switches: "CULL:QORDER" pairs, interleaved REPS times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for cq in ${COMBOS:-0:1 1:1 1:0 0:0}; do
    c=${cq%%:*}; q=${cq##*:}
    BOPX_VSD_CULL=$c BOPX_VSD_QORDER=$q timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 1 ${BENCH_ARGS} > gpurun_out/b.json 2> gpurun_out/b.err || { tail -30 gpurun_out/b.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/b.json'));print('cull %s qorder %s  vsd %.3f  value %d'%(sys.argv[1],sys.argv[2],d['kernels']['vsd']['ms'],d['value']))" $c $q
  done
done
