#!/bin/bash
# k_ortho Cholesky row broadcast through LDS: C5 tests + bench
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=gpurun_out/r3c
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_c5_gpu.py tests/test_structure_gpu.py > $O/c5n_tests.log 2>&1; rc=$?; tail -2 $O/c5n_tests.log; [ $rc = 0 ] || exit 1
for t in "ortho_min_tpb=2"; do
HH_TUNE=$t timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu --steps 5 --warmup 1 > $O/c5n_$t.log 2>&1 || exit 1
echo "$t $(tail -1 $O/c5n_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['config']['serial_step_ms'], [(k['kernel'][:10], round(k['total_ms'],1), k['launches']) for k in [r]+r['other_kernels']])")"
done
