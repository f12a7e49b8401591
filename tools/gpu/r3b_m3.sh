#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=gpurun_out/r3b
for cfg in c3 c2; do
it=20; [ $cfg = c2 ] && it=200
timeout -k 10 200 python -u tools/probe_knobs.py --config $cfg --iters $it "flatw_waves=11" "flatw_waves=8" > $O/m3_${cfg}_a.log 2>&1; echo "$cfg a rc=$?"; grep "\[1\]\|build" $O/m3_${cfg}_a.log
timeout -k 10 200 python -u tools/probe_knobs.py --config $cfg --iters $it --build flat_cols=0 "flatw_waves=11" > $O/m3_${cfg}_b.log 2>&1; echo "$cfg b rc=$?"; grep "\[1\]\|build" $O/m3_${cfg}_b.log
timeout -k 10 200 python -u tools/probe_knobs.py --config $cfg --iters $it --build flat_group=16 "flatw_waves=8" > $O/m3_${cfg}_c.log 2>&1; echo "$cfg c rc=$?"; grep "\[1\]\|build" $O/m3_${cfg}_c.log
done
