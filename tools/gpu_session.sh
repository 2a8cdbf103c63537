#!/bin/bash
# One parameterised GPU-box session (round 6; replaces the per-round one-off
# gpu_r0*_*.sh scripts). Steps, each under its own time limit, chained so the
# first failure ends the call:
#   TESTS=1      pytest -m gpu (PYTEST_ARGS narrows it, default the whole suite)
#   SMOKE=1      __graft_entry__.smoke()
#   BENCH=1      bench.py $BENCH_ARGS -> gpurun_out/bench_$TAG.json
#   PROFILE=1    rocprofv3 --kernel-trace --stats of the bench (no oracle legs)
#   PMC=1        the PMC passes of tools/pmc.sh -> gpurun_out/${TAG}_pmc.json
#   EXTRA="cmd"  one more command (its own limit: EXTRA_LIMIT seconds), before AB
#   AB="a b .."  interleaved A/B of libraries (paths relative to the repo; an
#                arm LIB:VAR=VAL,.. also sets that environment) on bench.py
#                $AB_ARGS, REPS rounds -> gpurun_out/ab_$TAG.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06}
fail() { echo "$1 failed"; tail -40 "$2"; exit 1; }
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${PYTEST_ARGS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || fail "gpu tests" gpurun_out/gpu_tests_$TAG.log
  tail -2 gpurun_out/gpu_tests_$TAG.log
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || fail smoke gpurun_out/smoke_$TAG.log
  tail -1 gpurun_out/smoke_$TAG.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || fail bench gpurun_out/bench_$TAG.err
  cut -c1-600 gpurun_out/bench_$TAG.json
fi
if [ -n "$PROFILE" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline --e2e-images 0 ${BENCH_ARGS} > gpurun_out/prof_$TAG.log 2>&1 || fail rocprof gpurun_out/prof_$TAG.log
  find gpurun_out/prof_$TAG -name "*kernel_stats*"
fi
if [ -n "$PMC" ]; then
  TAG=$TAG bash tools/pmc.sh "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" > gpurun_out/pmc_$TAG.log 2>&1 || fail pmc gpurun_out/pmc_$TAG.log
  tail -5 gpurun_out/pmc_$TAG.log
fi
if [ -n "$EXTRA" ]; then
  timeout -k 10 ${EXTRA_LIMIT:-600} bash -c "$EXTRA" > gpurun_out/extra_$TAG.log 2>&1 || fail extra gpurun_out/extra_$TAG.log
  tail -20 gpurun_out/extra_$TAG.log
fi
if [ -n "$AB" ]; then
  : > gpurun_out/ab_$TAG.txt
  for rep in $(seq ${REPS:-3}); do
    for arm in $AB; do
      # an arm: LIB or LIB:VAR=VALUE[,VAR=VALUE...] (environment of that arm)
      lib=${arm%%:*}; envs=""
      [ "$arm" != "$lib" ] && envs=$(echo "${arm#*:}" | tr ',' ' ')
      env $envs BOPX_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-images 0 ${AB_ARGS:---steps 5 --warmup 1} > gpurun_out/ab_one.json 2> gpurun_out/ab_one.err || fail "ab $arm" gpurun_out/ab_one.err
      python -c "import json,sys;d=json.load(open('gpurun_out/ab_one.json'));k=d['kernels'];print('%-50s rep %s %s value %.0f'%(sys.argv[1],sys.argv[2],' '.join('%s %.3f'%(n,v['ms']) for n,v in k.items() if isinstance(v,dict) and 'ms' in v),d['value']))" $arm $rep | tee -a gpurun_out/ab_$TAG.txt
    done
  done
fi
echo "session $TAG done"
