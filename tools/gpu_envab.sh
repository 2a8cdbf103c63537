#!/bin/bash
# A/B of environment settings on the default bench: each argument is one
# setting ("" = none), e.g. bash tools/gpu_envab.sh "" "BOPX_LAUNCH_ORDER=0".
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for setting in "$@"; do
  env $setting timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 ${BENCH_ARGS} > gpurun_out/var.json 2>gpurun_out/var.err || { tail gpurun_out/var.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/var.json'));print('[' + sys.argv[1] + ']', round(d['value']), {k:round(v['ms'],3) for k,v in d['kernels'].items()})" "$setting"
done
