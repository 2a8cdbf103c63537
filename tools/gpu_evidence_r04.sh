#!/bin/bash
# Round-4 evidence on one box: GPU tests + smoke + bench + rocprofv3 kernel
# stats (tools/gpu_round.sh), PMC passes of the same library on the default
# workload (tools/pmc.sh, summaries tagged with the library hash), then the
# bench again so its line carries the traffic of this build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04} PROFILE=1 bash tools/gpu_round.sh || exit 1
TAG=${TAG:-r04} bash tools/pmc.sh "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "GRBM_GUI_ACTIVE GRBM_COUNT" > gpurun_out/pmc_${TAG:-r04}.log 2>&1 || { tail -20 gpurun_out/pmc_${TAG:-r04}.log; exit 1; }
cp gpurun_out/${TAG:-r04}_pmc.json profiles/${TAG:-r04}_pmc.json
timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG:-r04}_traffic.json 2> gpurun_out/bench_${TAG:-r04}_traffic.err || { tail -20 gpurun_out/bench_${TAG:-r04}_traffic.err; exit 1; }
cat gpurun_out/bench_${TAG:-r04}_traffic.json
# multi-instance variant (shared renders): bench line + kernel stats
timeout -k 10 300 python bench.py --config 5 --tuples 20000 --no-cpu-baseline > gpurun_out/bench_${TAG:-r04}_config5.json 2> gpurun_out/bench_${TAG:-r04}_config5.err || { tail -20 gpurun_out/bench_${TAG:-r04}_config5.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG:-r04}_config5 -o run --output-format csv -- python3 bench.py --config 5 --tuples 20000 --no-cpu-baseline --steps 5 > gpurun_out/prof_${TAG:-r04}_config5.log 2>&1 || { tail -20 gpurun_out/prof_${TAG:-r04}_config5.log; exit 1; }
