#!/bin/bash
# MFMA experiment: configs[1] MSSD + MSPD with the exhaustive
# symmetry sweep (BOPX_SYM_PRUNE=0) on VALU FMAs vs v_mfma_f64_16x16x4_f64
# (BOPX_SYM_MFMA=1), interleaved, plus the pruned default; then one PMC pass of
# the MFMA build for its matrix-pipe busy cycles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for v in "0 0" "0 1" "2 0"; do
    set -- $v
    BOPX_SYM_PRUNE=$1 BOPX_SYM_MFMA=$2 timeout -k 10 200 python bench.py --config 1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/mf.json 2> gpurun_out/mf.err || { tail -20 gpurun_out/mf.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/mf.json'));print('prune %s mfma %s  mssd %.4f ms  mspd %.4f ms  value %d'%(sys.argv[1],sys.argv[2],d['kernels']['mssd']['ms'],d['kernels']['mspd']['ms'],d['value']))" $1 $2
  done
done
for v in "0 0" "0 1" "2 0"; do
  set -- $v
  BOPX_SYM_PRUNE=$1 BOPX_SYM_MFMA=$2 timeout -k 10 300 python bench.py --config 4 --tuples 20000 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/mf4.json 2> gpurun_out/mf4.err || { tail -20 gpurun_out/mf4.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/mf4.json'));print('configs[4] 20k: prune %s mfma %s  mssd %.4f ms  mspd %.4f ms'%(sys.argv[1],sys.argv[2],d['kernels']['mssd']['ms'],d['kernels']['mspd']['ms']))" $1 $2
done
for m in 0 1; do
  BOPX_SYM_PRUNE=0 BOPX_SYM_MFMA=$m timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-include-regex "k_sym" -d gpurun_out/mfpmc$m -o run --output-format csv -- python3 bench.py --config 1 --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/mfpmc$m.log 2>&1 || { echo "pmc $m failed"; tail -5 gpurun_out/mfpmc$m.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/mfma_pmc$m.json gpurun_out/mfpmc$m
done
