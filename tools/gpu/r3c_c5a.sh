#!/bin/bash
# C5 kernels rewritten (select / corr_norm / oe_center / colsum / diag_reduce) + fused split sum: tests, A/B bench
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=gpurun_out/r3c
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_c5_gpu.py tests/test_structure_gpu.py tests/test_fullsize_gpu.py > $O/c5a_tests.log 2>&1; rc=$?; tail -3 $O/c5a_tests.log; [ $rc = 0 ] || exit 1
for t in "cor_fuse=1" "cor_fuse=0"; do
HH_TUNE=$t timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu --steps 5 --warmup 1 > $O/c5a_$t.log 2>&1 || exit 1
echo "$t $(tail -1 $O/c5a_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['serial_step_ms'], d['config']['serial_phase_ms'])")"
done
