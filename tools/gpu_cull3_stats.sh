set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
L=$PWD/bop_toolkit_amd/lib/diag/libbopx_diag.so
BOPX_VSD_CULL=3 BOPX_LIB=$L BOPX_VSD_ABLATE=4 timeout -k 10 200 python tools/vsd_stats.py --tuples 3000 > gpurun_out/s3.txt 2>&1 || { tail gpurun_out/s3.txt; exit 1; }
BOPX_VSD_CULL=3 BOPX_LIB=$L BOPX_VSD_ABLATE=8 timeout -k 10 200 python tools/vsd_stats.py --tuples 3000 > gpurun_out/s3t.txt 2>&1 || { tail gpurun_out/s3t.txt; exit 1; }
BOPX_VSD_CULL=0 BOPX_LIB=$L BOPX_VSD_ABLATE=8 timeout -k 10 200 python tools/vsd_stats.py --tuples 3000 > gpurun_out/s0t.txt 2>&1 || { tail gpurun_out/s0t.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/s3.txt | head -14; paste gpurun_out/s0t.txt gpurun_out/s3t.txt | grep phase
COMBOS="product:0 old:0 product:3" REPS=2 bash tools/gpu_ab_libs.sh
