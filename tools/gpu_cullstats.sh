set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
L=$PWD/bop_toolkit_amd/lib/diag/libbopx_diag.so
BOPX_LIB=$L BOPX_VSD_ABLATE=4 timeout -k 10 200 python tools/vsd_stats.py --tuples 3000 > gpurun_out/cs_base.txt 2>&1 || { tail gpurun_out/cs_base.txt; exit 1; }
BOPX_VSD_CULL=1 BOPX_VSD_QORDER=0 BOPX_LIB=$L BOPX_VSD_ABLATE=4 timeout -k 10 200 python tools/vsd_stats.py --tuples 3000 > gpurun_out/cs_cull.txt 2>&1 || { tail gpurun_out/cs_cull.txt; exit 1; }
BOPX_VSD_CULL=2 BOPX_VSD_QORDER=0 BOPX_LIB=$L BOPX_VSD_ABLATE=4 timeout -k 10 200 python tools/vsd_stats.py --tuples 3000 > gpurun_out/cs_cull2.txt 2>&1 || { tail gpurun_out/cs_cull2.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/cs_base.txt gpurun_out/cs_cull.txt gpurun_out/cs_cull2.txt
