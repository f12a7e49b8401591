#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
O=gpurun_out/r3
timeout -k 10 300 python3 -u tools/pca_trace.py 1 --p 8 --coop 1 --reps 1 --debug 2 > $O/r3_c5e_phases.log 2>&1 || exit 1
grep "mode=0" $O/r3_c5e_phases.log | head -12
grep "mode=1\|mode=3" $O/r3_c5e_phases.log | head -4
for c in 1; do
timeout -k 10 300 python3 -u tools/pca_trace.py 1 21 --p 8 --coop $c --reps 3 > $O/r3_c5e_wall_$c.log 2>&1 || exit 1
grep Get_PCA $O/r3_c5e_wall_$c.log
done
