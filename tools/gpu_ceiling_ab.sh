set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in t6432trim3wg; do
  BOPX_LIB=$PWD/bop_toolkit_amd/lib/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "fused_vsd_bit_exact_lmo or ycbv_big or image_borders" -x -q --timeout 120 --timeout-method thread > gpurun_out/ceil_parity_$v.log 2>&1 || { tail -20 gpurun_out/ceil_parity_$v.log; exit 1; }
  tail -1 gpurun_out/ceil_parity_$v.log
done
REPS=2 BENCH_ARGS="--tuples 25000" bash tools/abrun.sh 2>&1 | tee gpurun_out/ceil_ab.txt
