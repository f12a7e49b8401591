#!/bin/bash
# C3 layout knobs (build-time) and run-time sweep knobs.  tools/gpu/r5j.sh outdir
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; mkdir -p $O
for b in "" "unit_entries=65536" "unit_entries=262144" "unit_entries=1048576" "flat_max=255" "flat_max=255,flat_cols=1" "tile_cost=0" "unit_lpt=0"; do
  echo "== build: $b"
  timeout -k 10 200 python3 -u tools/probe_knobs.py --config c3 --iters 20 --build "$b" "sweep_nb=2" "band_concurrent=1,conc_min_bytes=0" > $O/c3_b.log 2>&1 || { tail -20 $O/c3_b.log; exit 1; }
  grep -v amdgpu.ids $O/c3_b.log
done
