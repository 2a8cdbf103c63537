#!/bin/bash
# Device PNG decoder in the product path: the whole GPU suite + smoke on the
# new library, then the 100k-tuple e2e with the decoder A/B (warm runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_png.log 2>&1 || { tail -40 gpurun_out/gpu_tests_png.log; exit 1; }
tail -2 gpurun_out/gpu_tests_png.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_png.log 2>&1 || { tail -20 gpurun_out/smoke_png.log; exit 1; }
tail -2 gpurun_out/smoke_png.log
[ "${E2E:-1}" = 1 ] || exit 0
timeout -k 10 1000 python -u tools/e2e_bench.py --images 16667 --ab-depth > gpurun_out/e2e_png.json 2> gpurun_out/e2e_png.err || { tail -30 gpurun_out/e2e_png.err; exit 1; }
cat gpurun_out/e2e_png.json
rm -rf /tmp/bopx_e2e
