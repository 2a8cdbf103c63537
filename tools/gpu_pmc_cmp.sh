#!/bin/bash
# PMC counters of k_vsd for the product library and lib/variants/*.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for lib in bop_toolkit_amd/lib/libbopx.so bop_toolkit_amd/lib/variants/*.so; do
  tag=$(basename $lib .so)
  i=0
  for set in "SQC_ICACHE_MISSES SQC_ICACHE_REQ SQC_ICACHE_HITS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_IFETCH" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    BOPX_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_vsd" -d gpurun_out/cmp_${tag}_p$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --tuples 3000 > gpurun_out/cmp_${tag}_p$i.log 2>&1 || { echo "$tag pass $i failed"; tail -20 gpurun_out/cmp_${tag}_p$i.log; exit 1; }
  done
  python3 tools/pmc_summary.py gpurun_out/cmp_${tag}_pmc.json gpurun_out/cmp_${tag}_p* > /dev/null && echo "== $tag" && python3 -c "import json,sys;d=json.load(open(sys.argv[1]))['k_vsd'];[print('  %-22s %.4g'%(k,v)) for k,v in sorted(d.items())]" gpurun_out/cmp_${tag}_pmc.json
done
