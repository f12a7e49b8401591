#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=gpurun_out/r3b
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_c5_gpu.py -m gpu > $O/c5a_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/c5a_tests.log; [ $rc -eq 0 ] || exit $rc
for st in 8 4 12; do
HH_C5_STREAMS=$st timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu --steps 5 --warmup 1 > $O/c5a_s$st.log 2>&1; echo "streams $st rc=$?"; tail -1 $O/c5a_s$st.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['config']['serial_step_ms'], r['kernel'], r['total_ms'], [(o['kernel'][:12], o['total_ms']) for o in r['other_kernels']])"
done
