#!/bin/bash
# serial (one stream) Get_PCA wall and kernel trace, k_ortho on / off
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
O=gpurun_out/r3
for c in 0 1; do
timeout -k 10 300 python3 -u tools/pca_trace.py 1 21 --p 8 --coop $c --reps 4 > $O/r3_c5d_wall_$c.log 2>&1 || exit 1
grep Get_PCA $O/r3_c5d_wall_$c.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c5dprof$c -o c5 -- python3 -u $GRAFT_REPO_ROOT/tools/pca_trace.py 1 --p 8 --coop $c --reps 2 > $GRAFT_REPO_ROOT/$O/r3_c5d_prof_$c.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
done
echo ok
