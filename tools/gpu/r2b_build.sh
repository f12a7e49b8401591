#!/bin/bash
# device build with pipelined row passes: build tests, drop-in / e2e lines with phase times
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/build && export TMPDIR=/tmp
O=gpurun_out/build
timeout -k 10 600 python -u -m pytest tests/test_build_gpu.py tests/test_pairs_gpu.py tests/test_gw_sparse_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
HH_BUILD_DEBUG=1 timeout -k 10 300 python3 -u bench.py --config dropin --steps 3 --warmup 1 --no-cpu > $O/dropin.log 2>&1 || exit 1
grep -E "pass|sort|keys|check|plan" $O/dropin.log | tail -12
tail -1 $O/dropin.log | cut -c1-400
HH_BUILD_DEBUG=1 timeout -k 10 300 python3 -u bench.py --config e2e --steps 3 --warmup 1 --no-cpu > $O/e2e.log 2>&1 || exit 1
grep -E "pass|sort" $O/e2e.log | tail -6
tail -1 $O/e2e.log | cut -c1-400
echo done
