#!/bin/bash
# rocprofv3 PMC passes over a short bench run (kernel-trace + counters only; no
# sys/runtime trace domains). Usage: TAG=.. bash tools/pmc.sh "<counters>" ["<counters>" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-pmc}
i=0
for set in "$@"; do
  i=$((i+1))
  mkdir -p gpurun_out/${TAG}_p$i
  BOPX_BENCH_META=gpurun_out/${TAG}_p$i/meta.json timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "${KREGEX:-k_vsd|k_sym_error}" -d gpurun_out/${TAG}_p$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline --e2e-images 0 --steps 1 --warmup 0 ${BENCH_ARGS:-} > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -20 gpurun_out/${TAG}_p$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc.json gpurun_out/${TAG}_p*
