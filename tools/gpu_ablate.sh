#!/bin/bash
# k_vsd timing ablations on the diag build (BOPX_VSD_ABLATE bits; results are
# wrong by design for bits 1, 2, 16): kernel ms from bench.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for ab in ${ABL:-0 16 0 16}; do
BOPX_LIB=$PWD/bop_toolkit_amd/lib/diag/libbopx_diag.so BOPX_VSD_ABLATE=$ab timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/b.json 2> gpurun_out/b.err || { tail -30 gpurun_out/b.err; exit 1; }
python -c "import json,sys;d=json.load(open('gpurun_out/b.json'));print('ablate',sys.argv[1],'cull',sys.argv[2],{k:round(v['ms'],3) for k,v in d['kernels'].items()})" $ab ${BOPX_VSD_CULL:-1}
done
