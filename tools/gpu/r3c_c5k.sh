#!/bin/bash
# C5 host threads / streams A/B at the current build
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=gpurun_out/r3c
for st in 16 8 12; do
HH_C5_STREAMS=$st timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu --steps 5 --warmup 1 > $O/c5k_s$st.log 2>&1 || exit 1
echo "streams $st $(tail -1 $O/c5k_s$st.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['serial_step_ms'])")"
done
