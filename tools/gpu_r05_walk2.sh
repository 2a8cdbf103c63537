#!/bin/bash
# k_vsd two-row walk items: parity (the VSD suites + a fuzz subset) on the new
# build, then an interleaved A/B of k_vsd ms against lib/variants/vsd_prev.so
# on configs 3 / 4 / 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05w2}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shared.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_parity_${TAG}.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/gpu_parity_${TAG}.log; exit 1; }
tail -1 gpurun_out/gpu_parity_${TAG}.log
BOPX_FUZZ_CASES=${FUZZ:-200} timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q --timeout 380 --timeout-method thread > gpurun_out/gpu_fuzz_${TAG}.log 2>&1 || { echo "fuzz failed"; tail -30 gpurun_out/gpu_fuzz_${TAG}.log; exit 1; }
tail -1 gpurun_out/gpu_fuzz_${TAG}.log
for cfg in ${CFGS:-3 4 5}; do
  for rep in $(seq ${REPS:-3}); do
    for v in prev new; do
      lib=$PWD/bop_toolkit_amd/lib/libbopx.so
      [ $v = prev ] && lib=$PWD/bop_toolkit_amd/lib/variants/vsd_prev.so
      BOPX_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --e2e-images 0 --steps ${STEPS:-5} --warmup 1 > gpurun_out/w2_${TAG}_${cfg}_${v}_$rep.json 2> gpurun_out/w2_${TAG}.err || { tail -30 gpurun_out/w2_${TAG}.err; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print('cfg %s %-5s rep %s  vsd %.3f  value %d'%(sys.argv[2],sys.argv[3],sys.argv[4],d['kernels']['vsd']['ms'],d['value']))" gpurun_out/w2_${TAG}_${cfg}_${v}_$rep.json $cfg $v $rep
    done
  done
done
