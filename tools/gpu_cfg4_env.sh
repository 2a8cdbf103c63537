#!/bin/bash
# Runtime-toggle sweep on the T-LESS-like shard (configs[4]); defaults were
# tuned on configs[3]. Same box, interleaved, REPS repetitions.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for combo in "default" "BOPX_VSD_QORDER=0" "BOPX_SYM_PRUNE=4" "BOPX_SYM_PRUNE=8" "BOPX_MESHLET_CURVE=morton" "BOPX_VSD_CULL=3"; do
    envs=""; [ "$combo" != default ] && envs="$combo"
    env $envs timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -30 gpurun_out/c4.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/c4.json'));print('%-22s %s value %d'%(sys.argv[1], {k:round(v['ms'],3) for k,v in d['kernels'].items()}, d['value']))" "$combo"
  done
done
