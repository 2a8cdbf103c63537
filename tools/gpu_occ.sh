set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for d in 0 50000 0 50000; do
BOPX_VSD_DYNLDS=$d BOPX_VSD_CULL=0 BOPX_LIB=$PWD/bop_toolkit_amd/lib/diag/libbopx_diag.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/b.json 2> gpurun_out/b.err || { tail -30 gpurun_out/b.err; exit 1; }
python -c "import json,sys;d=json.load(open('gpurun_out/b.json'));print('dynlds',sys.argv[1],{k:round(v['ms'],3) for k,v in d['kernels'].items()})" $d
done
