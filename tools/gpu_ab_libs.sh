#!/bin/bash
# Same-box interleaved A/B of "LIB:CULL" pairs (LIB = product | variant name).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for lc in ${COMBOS}; do
    l=${lc%%:*}; c=${lc##*:}
    lib=$PWD/bop_toolkit_amd/lib/libbopx.so; [ "$l" != product ] && lib=$PWD/bop_toolkit_amd/lib/variants/$l.so
    BOPX_VSD_CULL=$c BOPX_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 1 ${BENCH_ARGS} > gpurun_out/b.json 2> gpurun_out/b.err || { tail -30 gpurun_out/b.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/b.json'));print('%-10s cull %s  vsd %.3f  mssd %.3f  mspd %.3f  value %d'%(sys.argv[1],sys.argv[2],d['kernels']['vsd']['ms'],d['kernels']['mssd']['ms'],d['kernels']['mspd']['ms'],d['value']))" $l $c
  done
done
