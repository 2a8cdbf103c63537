#!/bin/bash
# Full round evidence: parity tests, smoke, bench, rocprofv3 kernel stats, PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r01}
PROFILE=1 TAG=$TAG bash tools/gpu_round.sh || exit 1
TAG=$TAG BENCH_ARGS="--config 3" bash tools/pmc.sh FETCH_SIZE WRITE_SIZE \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY" > gpurun_out/pmc_${TAG}.log 2>&1 || { tail -20 gpurun_out/pmc_${TAG}.log; exit 1; }
tail -40 gpurun_out/pmc_${TAG}.log
