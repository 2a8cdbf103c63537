set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
L=$PWD/bop_toolkit_amd/lib/diag/libbopx_diag.so
BOPX_LIB=$L BOPX_VSD_ABLATE=4 timeout -k 10 200 python tools/vsd_stats.py --tuples 3000 > gpurun_out/stats4.txt 2>&1 || { tail gpurun_out/stats4.txt; exit 1; }
BOPX_LIB=$L BOPX_VSD_ABLATE=8 timeout -k 10 200 python tools/vsd_stats.py --tuples 3000 > gpurun_out/stats8.txt 2>&1 || { tail gpurun_out/stats8.txt; exit 1; }
cat gpurun_out/stats4.txt gpurun_out/stats8.txt | grep -v amdgpu.ids
