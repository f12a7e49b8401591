#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
O=gpurun_out/r3b
timeout -k 10 200 python3 -u tools/probe_uband.py 14637 1 > $O/ub4_probe.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids $O/ub4_probe.log | head -40
timeout -k 10 200 python3 -u tools/probe_uband.py 14637 0 > $O/ub4_probe8.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids $O/ub4_probe8.log | head -40
