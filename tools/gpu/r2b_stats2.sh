#!/bin/bash
# big-mode tile sums fused into k_marg: ICE / dist / full-size tests, C4 / C3 A/B (fuse_stats -1 vs 0)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/st2 && export TMPDIR=/tmp
O=gpurun_out/st2
timeout -k 10 700 python -u -m pytest tests/test_ice_gpu.py tests/test_dist_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/probe_knobs.py --iters 20 "fuse_stats=-1" "fuse_stats=0" 2>&1 | grep sweep | sed 's/^/c4: /' >> $O/ab.log || exit 1
timeout -k 10 200 python3 -u tools/probe_knobs.py --config c3 --iters 200 "fuse_stats=-1" "fuse_stats=0" 2>&1 | grep sweep | sed 's/^/c3: /' >> $O/ab.log || exit 1
cat $O/ab.log
