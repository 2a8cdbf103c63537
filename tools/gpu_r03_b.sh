#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shared.py -x -q --timeout 200 --timeout-method thread -k "mfma or shared" > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
bash tools/gpu_mfma.sh 2>&1 | grep -E "prune|MFMA_BUSY|k_sym|failed" || exit 1
timeout -k 10 300 python bench.py --config 5 --tuples 20000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b5.json 2> gpurun_out/b5.err || { tail gpurun_out/b5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b5.json'));print('config5', d['kernels']['vsd']['ms'], d['kernels']['vsd_fused_per_tuple']['ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python3 bench.py --config 5 --tuples 20000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof5.log 2>&1 || exit 1
find gpurun_out/prof5 -name "*kernel_stats.csv" | xargs cat | cut -c1-110 | head -6
