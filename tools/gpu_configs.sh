#!/bin/bash
# bench.py on every BASELINE.json configuration (1 GPU) -> gpurun_out/cfg/configN.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/cfg; export TMPDIR=/tmp
for c in 0 1 2 3 4; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 1 > gpurun_out/cfg/config$c.json 2> gpurun_out/cfg/config$c.err || { tail -20 gpurun_out/cfg/config$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/cfg/config$c.json'));print($c, round(d['value']), {k:round(v['ms'],2) for k,v in d['kernels'].items()})"
done
