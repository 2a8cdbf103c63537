#!/bin/bash
# VALU / SALU / LDS instruction counts of k_vsd per diag ablation (bits: 1 no raster,
# 2 no pixel pass, 32 no row walk, 64 no set-up + walk; results wrong by design).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/bop_toolkit_amd/lib/diag/libbopx_diag.so
for ab in ${ABL:-0 1 2 32 64}; do
  BOPX_LIB=$L BOPX_VSD_ABLATE=$ab timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "k_vsd" -d gpurun_out/abp_$ab -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --tuples 3000 > gpurun_out/abp_$ab.log 2>&1 || { echo "ablate $ab failed"; tail -20 gpurun_out/abp_$ab.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/abp_${ab}.json gpurun_out/abp_$ab > /dev/null && python3 -c "import json,sys;d=json.load(open(sys.argv[1]))['k_vsd'];print('ablate %-3s'%sys.argv[2], ' '.join('%s %.4g'%(k.replace('SQ_',''),v/3000) for k,v in sorted(d.items()) if k.startswith('SQ')))" gpurun_out/abp_${ab}.json $ab
done
