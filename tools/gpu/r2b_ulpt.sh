#!/bin/bash
# unit launch lists by cost class (unit_lpt, build knob): shard / whole-C4 / C3 / C2 A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/ulpt && export TMPDIR=/tmp
O=gpurun_out/ulpt
for x in 1 0 1 0; do
  for k in 3 7 0; do timeout -k 10 200 python3 -u tools/probe_knobs.py --shard $k/8 --iters 30 --build unit_lpt=$x "band_lpt=1" 2>&1 | grep "shard iter" | sed "s/^/unit_lpt=$x shard $k: /" >> $O/ab.log || exit 1; done
done
for x in 1 0 1 0; do
  timeout -k 10 200 python3 -u tools/probe_knobs.py --iters 20 --build unit_lpt=$x "band_lpt=1" 2>&1 | grep "sweep" | sed "s/^/unit_lpt=$x c4: /" >> $O/ab.log || exit 1
  for c in c3 c2; do timeout -k 10 200 python3 -u tools/probe_knobs.py --config $c --iters 200 --build unit_lpt=$x "band_lpt=1" 2>&1 | grep "sweep" | sed "s/^/unit_lpt=$x $c: /" >> $O/ab.log || exit 1; done
done
sort $O/ab.log
