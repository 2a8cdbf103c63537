#!/bin/bash
# GPU parity tests, k_vsd workload counters (diag build), then the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
BOPX_LIB=$PWD/bop_toolkit_amd/lib/diag/libbopx_diag.so BOPX_VSD_ABLATE=4 timeout -k 10 200 python tools/vsd_stats.py --tuples 3000 > gpurun_out/stats4.txt 2>&1 || { tail gpurun_out/stats4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stats4.txt | head -11
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(round(d['value']), {k:round(v['ms'],3) for k,v in d['kernels'].items()})"
