#!/bin/bash
# Same-box interleaved A/B of environment settings (each argument one setting,
# "" = none), REPS rounds; prints k_vsd ms and the step throughput.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for setting in "$@"; do
    env $setting timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 1 ${BENCH_ARGS} > gpurun_out/b.json 2> gpurun_out/b.err || { tail -30 gpurun_out/b.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/b.json'));print('%-28s vsd %.3f  mssd %.3f  mspd %.3f  value %d'%(sys.argv[1],d['kernels']['vsd']['ms'],d['kernels']['mssd']['ms'],d['kernels']['mspd']['ms'],d['value']))" "[$setting]"
  done
done
