#!/bin/bash
# LDS / issue counters of k_vsd (one rocprofv3 --pmc pass per counter set).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-lds}
i=0
for set in "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_vsd" -d gpurun_out/${TAG}_p$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --tuples 3000 > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -20 gpurun_out/${TAG}_p$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc.json gpurun_out/${TAG}_p* && cat gpurun_out/${TAG}_pmc.json
