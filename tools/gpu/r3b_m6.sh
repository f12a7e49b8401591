#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
timeout -k 10 200 python -u tools/probe_filters.py c3 > gpurun_out/r3b/m6_c3_filters.log 2>&1; echo "rc=$?"; grep "\[" gpurun_out/r3b/m6_c3_filters.log
timeout -k 10 200 python -u tools/probe_filters.py c2 > gpurun_out/r3b/m6_c2_filters.log 2>&1; echo "rc=$?"; grep "\[" gpurun_out/r3b/m6_c2_filters.log
