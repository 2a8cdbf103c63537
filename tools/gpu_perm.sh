#!/bin/bash
# k_vsd launch-order experiments (same box): device order (cost classes +
# slot, the product), no order, and host-side permutations of the bench tuples.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
run() { env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/b.json 2> gpurun_out/b.err || { tail -30 gpurun_out/b.err; exit 1; }
python -c "import json,sys;d=json.load(open('gpurun_out/b.json'));print('%-48s vsd %.3f mssd %.3f mspd %.3f'%(sys.argv[1],d['kernels']['vsd']['ms'],d['kernels']['mssd']['ms'],d['kernels']['mspd']['ms']))" "$*"; }
for rep in 1 2; do
run BOPX_X=product
run BOPX_LIB=$PWD/bop_toolkit_amd/lib/variants/base.so
run BOPX_LAUNCH_ORDER=0 BOPX_BENCH_PERM=lptobj8
done
