#!/bin/bash
# Same-box interleaved A/B of every library in lib/variants (and the product
# one) on a 25k-tuple configs[3] batch (tools/abrun.sh), output to
# gpurun_out/${TAG}_ab.txt. Optional parity subset of a variant first (CHECK=name).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${CHECK}; do
  BOPX_LIB=$PWD/bop_toolkit_amd/lib/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shared.py -m gpu -k "${CHECK_K:-fused or shared}" -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_parity_$v.log 2>&1 || { tail -20 gpurun_out/${TAG}_parity_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/${TAG}_parity_$v.log)"
done
REPS=${REPS:-3} BENCH_ARGS="${BENCH_ARGS:---tuples 25000}" bash tools/abrun.sh 2>&1 | tee gpurun_out/${TAG}_ab.txt
