#!/bin/bash
# C5 chromosome scheduling over the stream workers: one largest-first queue vs round-robin lanes
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=gpurun_out/r3c
for sc in queue static queue; do
HH_C5_SCHED=$sc timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu --steps 5 --warmup 1 > $O/c5sched_$sc.log 2>&1 || exit 1
echo "$sc $(tail -1 $O/c5sched_$sc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['serial_step_ms'])")"
done
