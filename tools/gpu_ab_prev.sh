#!/bin/bash
# Same-box interleaved A/B: the product library against a variant library
# (bop_toolkit_amd/lib/variants/$VARIANT.so, e.g. the previous commit's build),
# runtime toggles left at their defaults. BENCH_ARGS selects the workload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in $(seq ${REPS:-3}); do
  for l in product ${VARIANT}; do
    lib=$PWD/bop_toolkit_amd/lib/libbopx.so; [ "$l" != product ] && lib=$PWD/bop_toolkit_amd/lib/variants/$l.so
    BOPX_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -30 gpurun_out/ab.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));print('%-10s %s value %d'%(sys.argv[1], {k:round(v['ms'],3) for k,v in d['kernels'].items()}, d['value']))" $l
  done
done
