#!/bin/bash
# C4 N-GPU shards (payload partition) under several hh_tune settings, one
# probe_shards run each: tools/gpu/shard_knobs.sh outdir world "k=v,..." "k=v,..." ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
O=gpurun_out/$1; W=$2; shift 2; mkdir -p $O
i=0
for spec in "$@"; do
  i=$((i+1))
  HH_TUNE="$spec" timeout -k 10 300 python3 -u tools/probe_shards.py $W 0 > $O/knobs_$i.log 2>&1 || { echo "$spec failed"; tail -3 $O/knobs_$i.log; exit 1; }
  echo "[$spec] $(grep "max " $O/knobs_$i.log | tail -1)"
done
