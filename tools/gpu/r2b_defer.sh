#!/bin/bash
# flat kernel: compact-sum merge deferred past the next tile's barrier (flat_defer 1) vs round-1 order (0)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/defer && export TMPDIR=/tmp
O=gpurun_out/defer
timeout -k 10 600 python -u -m pytest tests/test_ice_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/probe_knobs.py --iters 20 "flat_defer=1" "flat_defer=0" 2>&1 | grep sweep | sed 's/^/c4: /' >> $O/ab.log || exit 1
timeout -k 10 200 python3 -u tools/probe_knobs.py --iters 20 "conc_min_bytes=1000000000000,flat_defer=1" "conc_min_bytes=1000000000000,flat_defer=0" 2>&1 | grep sweep | sed 's/^/c4 1-stream: /' >> $O/ab.log || exit 1
timeout -k 10 200 python3 -u tools/probe_knobs.py --config c3 --iters 200 "flat_defer=1" "flat_defer=0" 2>&1 | grep sweep | sed 's/^/c3: /' >> $O/ab.log || exit 1
timeout -k 10 200 python3 -u tools/probe_knobs.py --config c2 --iters 200 "flat_defer=1" "flat_defer=0" 2>&1 | grep sweep | sed 's/^/c2: /' >> $O/ab.log || exit 1
for k in 0 7; do timeout -k 10 200 python3 -u tools/probe_knobs.py --shard $k/8 --iters 30 "flat_defer=1" "flat_defer=0" 2>&1 | grep "shard iter" | sed "s/^/shard $k: /" >> $O/ab.log || exit 1; done
cat $O/ab.log
