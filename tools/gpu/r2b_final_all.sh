#!/bin/bash
# GPU suite + smoke, then the measurement set (tools/gpu/r2b_final.sh) of commit $1
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/final && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/r2b_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/final/r2b_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/r2b_smoke.log 2>&1 || exit 1
echo "smoke ok"
bash tools/gpu/r2b_final.sh "$1"
