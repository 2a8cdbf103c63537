set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for c in ${CULLS:-1 0 2 1 0 2}; do
BOPX_VSD_CULL=$c timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/b.json 2> gpurun_out/b.err || { tail -30 gpurun_out/b.err; exit 1; }
python -c "import json,sys;d=json.load(open('gpurun_out/b.json'));print('cull',sys.argv[1],round(d['value']), {k:round(v['ms'],3) for k,v in d['kernels'].items()})" $c
done
for c in ${PCULLS:-1 0}; do
BOPX_VSD_CULL=$c BOPX_LIB=$PWD/bop_toolkit_amd/lib/diag/libbopx_diag.so BOPX_VSD_ABLATE=8 timeout -k 10 200 python tools/vsd_stats.py --tuples 3000 > gpurun_out/stats8.txt 2>&1 || { tail gpurun_out/stats8.txt; exit 1; }
echo "== phases cull=$c"; grep phase gpurun_out/stats8.txt
done
