#!/bin/bash
# Round 4: k_vsd_pair variants on the multi-instance configs[5] and the
# per-symmetry-class MSSD / MSPD times (tools/sym_classes.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
REPS=3 BENCH_ARGS="--config 5 --tuples 20000" bash tools/abrun.sh 2>&1 | tee gpurun_out/ab3_config5.txt || exit 1
timeout -k 10 300 python tools/sym_classes.py --config 3 > gpurun_out/sym_classes_c3.txt 2> gpurun_out/sym_classes_c3.err || { tail -20 gpurun_out/sym_classes_c3.err; exit 1; }
cat gpurun_out/sym_classes_c3.txt
timeout -k 10 300 python tools/sym_classes.py --config 4 --n 2000 > gpurun_out/sym_classes_c4.txt 2> gpurun_out/sym_classes_c4.err || { tail -20 gpurun_out/sym_classes_c4.err; exit 1; }
cat gpurun_out/sym_classes_c4.txt
