set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r02d} PROFILE=1 bash tools/gpu_round.sh || exit 1
TAG=${TAG:-r02d} BENCH_ARGS=" " bash tools/pmc.sh "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" > gpurun_out/pmc_${TAG:-r02d}.log 2>&1 || { tail -20 gpurun_out/pmc_${TAG:-r02d}.log; exit 1; }
tail -40 gpurun_out/pmc_${TAG:-r02d}.log
