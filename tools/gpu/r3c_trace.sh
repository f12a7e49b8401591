#!/bin/bash
# inlined k_ortho: per-phase timestamps (pca_debug 2) on chr1, and Get_PCA wall per chromosome
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=gpurun_out/r3c
timeout -k 10 300 python3 -u tools/pca_trace.py 1 --p 8 --debug 2 > $O/trace_chr1.log 2>&1 || exit 1
grep -m3 "mode=0 nb=7\|mode=0 nb=1 " $O/trace_chr1.log | cut -c1-250
tail -2 $O/trace_chr1.log | cut -c1-200
timeout -k 10 300 python3 -u tools/pca_trace.py 1 21 --p 8 --debug 0 --reps 3 > $O/trace_wall.log 2>&1 || exit 1
cat $O/trace_wall.log | cut -c1-200
