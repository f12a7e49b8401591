#!/bin/bash
# uband rule for mid-size matrices (C3, C4 haploid, cis) and the TwoStep
# genome line's kernel profile.   tools/gpu/r5g.sh outdir
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; mkdir -p $O
for cfg in c3 c4h; do
timeout -k 10 300 python3 -u tools/probe_knobs.py --config $cfg --iters 20 "uband=0" "uband=2" "uband=2,conc_ub_min_bytes=0" "uband=0,conc_min_bytes=0" > $O/${cfg}_knobs.log 2>&1 || { tail -20 $O/${cfg}_knobs.log; exit 1; }
cat $O/${cfg}_knobs.log
done
bash tools/gpu/prof_line.sh $1 twostep_genome --steps 5 --warmup 1
