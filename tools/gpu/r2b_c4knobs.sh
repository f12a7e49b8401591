#!/bin/bash
# C4 build knobs re-checked on the final kernels: unit size, flat_max
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/c4k && export TMPDIR=/tmp
O=gpurun_out/c4k
for b in "" "unit_entries=262144" "flat_max=48" "flat_max=96" ""; do
  timeout -k 10 200 python3 -u tools/probe_knobs.py --iters 20 ${b:+--build $b} "band_lpt=1" 2>&1 | grep sweep | sed "s/^/[${b:-default}] /" >> $O/ab.log || exit 1
done
cat $O/ab.log
