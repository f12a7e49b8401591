#!/bin/bash
# flat column-group size on C4 (bias staging per group vs tail): sweep times
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=gpurun_out/r3c
timeout -k 10 400 python3 -u tools/probe_knobs.py --iters 20 "flat_group=0" "flat_group=64" "flat_group=88" "flat_group=0" > $O/fg_probe.log 2>&1 || exit 1
grep -v "^$" $O/fg_probe.log | tail -8 | cut -c1-200
