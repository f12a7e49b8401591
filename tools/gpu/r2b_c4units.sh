#!/bin/bash
# whole-C4 unit size (build knob unit_entries; auto = words / 4096 = 446 K words) and the N = 2 shard
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/c4u && export TMPDIR=/tmp
O=gpurun_out/c4u
for b in "" "unit_entries=196608" "unit_entries=262144" "unit_entries=327680" "unit_entries=262144,tile_cost=0" ""; do
  timeout -k 10 200 python3 -u tools/probe_knobs.py --iters 20 ${b:+--build $b} "band_lpt=1" 2>&1 | grep sweep | sed "s/^/c4 [${b:-default}] /" >> $O/ab.log || exit 1
done
for b in "" "unit_entries=262144" ""; do
  timeout -k 10 200 python3 -u tools/probe_knobs.py --shard 0/2 --iters 20 ${b:+--build $b} "band_lpt=1" 2>&1 | grep "shard iter" | sed "s/^/shard 0\/2 [${b:-default}] /" >> $O/ab.log || exit 1
done
cat $O/ab.log
