#!/bin/bash
# C2 single-launch sweep vs unit size (build knob unit_entries; 0 = auto = 32768 words at C2)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/c2u && export TMPDIR=/tmp
O=gpurun_out/c2u
for ue in 0 49152 65536 98304 24576 0; do
  timeout -k 10 200 python3 -u tools/probe_knobs.py --config c2 --iters 300 --build unit_entries=$ue "band_lpt=1" 2>&1 | grep sweep | sed "s/^/unit_entries=$ue: /" >> $O/ab.log || exit 1
done
for tc in 0 16384 65536; do
  timeout -k 10 200 python3 -u tools/probe_knobs.py --config c2 --iters 300 --build tile_cost=$tc "band_lpt=1" 2>&1 | grep sweep | sed "s/^/tile_cost=$tc: /" >> $O/ab.log || exit 1
done
cat $O/ab.log
