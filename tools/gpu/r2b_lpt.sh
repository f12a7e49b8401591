#!/bin/bash
# band chunks heaviest-first: ICE tests, shard / whole-C4 A/B, N=8 shard probe
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/lpt && export TMPDIR=/tmp
O=gpurun_out/lpt
timeout -k 10 600 python -u -m pytest tests/test_ice_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for k in 3 7 0; do timeout -k 10 200 python3 -u tools/probe_knobs.py --shard $k/8 --iters 30 "band_lpt=1" "band_lpt=0" >> $O/shard_ab.log 2>&1 || exit 1; done
grep "shard iter" $O/shard_ab.log
timeout -k 10 300 python3 -u tools/probe_knobs.py --iters 20 "band_lpt=1" "band_lpt=0" > $O/c4_ab.log 2>&1 || exit 1
grep -v "^{" $O/c4_ab.log | tail -6
HH_TUNE=band_lpt=1 timeout -k 10 400 python3 -u tools/probe_shards.py 8 1 > $O/probe_shards8.log 2>&1 || exit 1
tail -3 $O/probe_shards8.log
echo done
