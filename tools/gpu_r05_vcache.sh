#!/bin/bash
# k_vsd staged-vertex cache: full GPU suite with the cache on (default), then a
# same-box interleaved A/B of k_vsd ms: previous library (lib/variants/vsd_prev.so),
# the product library with BOPX_VSD_VCACHE=1 and =0, on the bench workload
# (configs[3]) and on configs[4] / configs[5].
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05v}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_parity_${TAG}.log 2>&1 || { echo "parity tests failed"; tail -30 gpurun_out/gpu_parity_${TAG}.log; exit 1; }
tail -1 gpurun_out/gpu_parity_${TAG}.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_${TAG}.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_${TAG}.log; exit 1; }
tail -2 gpurun_out/gpu_tests_${TAG}.log
for cfg in ${CFGS:-3 4 5}; do
  for rep in $(seq ${REPS:-3}); do
    for v in prev vc1 vc0; do
      lib=$PWD/bop_toolkit_amd/lib/libbopx.so; vc=1
      [ $v = prev ] && lib=$PWD/bop_toolkit_amd/lib/variants/vsd_prev.so
      [ $v = vc0 ] && vc=0
      BOPX_VSD_VCACHE=$vc BOPX_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --e2e-images 0 --steps ${STEPS:-5} --warmup 1 > gpurun_out/vc_${TAG}_${cfg}_${v}_$rep.json 2> gpurun_out/vc_${TAG}.err || { tail -30 gpurun_out/vc_${TAG}.err; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print('cfg %s %-5s rep %s  vsd %.3f  value %d'%(sys.argv[2],sys.argv[3],sys.argv[4],d['kernels']['vsd']['ms'],d['value']))" gpurun_out/vc_${TAG}_${cfg}_${v}_$rep.json $cfg $v $rep
    done
  done
done
