#!/bin/bash
# C4 row shards of the N-GPU partitions swept one at a time on this GPU, per
# kernel (HIP-event registry, one stream), the whole matrix first.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
O=gpurun_out/${1:-shards}; mkdir -p $O
HH_TUNE=band_concurrent=0 timeout -k 10 600 python3 -u tools/probe_shards.py ${2:-1,2,4,8} ${3:-0} > $O/shards.log 2>&1
