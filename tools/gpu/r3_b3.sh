#!/bin/bash
# GW merge restructure + a C5 PCA per-cycle trace + C4 sweep kernel profile (one stream)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
O=gpurun_out/r3
bash tools/gpu/r3_gwm.sh || exit 1
timeout -k 10 300 python3 -u tools/pca_trace.py 21 1 --p 8 > $O/r3_pca_trace.log 2>&1 || exit 1
tail -3 $O/r3_pca_trace.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c4prof -o c4 -- python3 -u $GRAFT_REPO_ROOT/tools/probe_knobs.py --iters 10 "band_concurrent=0" > $GRAFT_REPO_ROOT/$O/r3_c4_prof.log 2>&1 || exit 1
echo c4 prof ok
