#!/bin/bash
# Round-5 first box: the round-4 evidence chain on HEAD (GPU tests, smoke,
# bench, rocprofv3 kernel stats, PMC passes keyed on the code objects, bench
# again with traffic, configs[5]) and the diag build's wave-level loop trip
# counts on the full configs[3] job (tools/isa_census.py input).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05s}
BOPX_LIB=$PWD/bop_toolkit_amd/lib/diag/libbopx_diag.so BOPX_VSD_ABLATE=4 BOPX_VSD_STATS_JSON=gpurun_out/census_counts_${TAG}.json timeout -k 10 300 python tools/vsd_stats.py --tuples 100000 > gpurun_out/diag_census_${TAG}.log 2>&1 || { tail -20 gpurun_out/diag_census_${TAG}.log; exit 1; }
grep -E "per tuple" gpurun_out/diag_census_${TAG}.log
TAG=$TAG bash tools/gpu_evidence_r04.sh
# end to end at the metric's scale: cold run, then warm A/B of per-scene and
# grouped GPU depth-decode launches
timeout -k 10 420 python tools/e2e_bench.py --images 16667 --ab-depth --ab-group > gpurun_out/e2e_100k_${TAG}.json 2> gpurun_out/e2e_100k_${TAG}.err || { tail -20 gpurun_out/e2e_100k_${TAG}.err; exit 1; }
cat gpurun_out/e2e_100k_${TAG}.json
