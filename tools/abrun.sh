#!/bin/bash
# Same-box A/B: k_vsd ms of every library in lib/variants (and the product one)
# under each BOPX_VSD_CULL setting, interleaved REPS times (box-to-box clock
# differences make cross-call comparisons unreliable).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for lib in bop_toolkit_amd/lib/libbopx.so bop_toolkit_amd/lib/variants/*.so; do
    for c in ${CULLS:--1}; do
      BOPX_VSD_CULL=$c BOPX_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 1 ${BENCH_ARGS} > gpurun_out/b.json 2> gpurun_out/b.err || { tail -30 gpurun_out/b.err; exit 1; }
      python -c "import json,sys;d=json.load(open('gpurun_out/b.json'));print('%-16s cull %s  vsd %.3f  mssd %.3f  mspd %.3f  value %d'%(sys.argv[1],sys.argv[2],d['kernels']['vsd']['ms'],d['kernels']['mssd']['ms'],d['kernels']['mspd']['ms'],d['value']))" $(basename $lib .so) $c
    done
  done
done
