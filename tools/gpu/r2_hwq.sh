#!/bin/bash
# C5 with 8 host streams: hardware queues 4 (default) vs 8
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/hwq
timeout -k 10 300 python3 -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu > gpurun_out/hwq/c5_q4.log 2>&1 || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu > gpurun_out/hwq/c5_q8.log 2>&1 || exit 1
GPU_MAX_HW_QUEUES=8 HH_C5_STREAMS=16 timeout -k 10 300 python3 -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu > gpurun_out/hwq/c5_q8s16.log 2>&1 || exit 1
for f in c5_q4 c5_q8 c5_q8s16; do tail -1 gpurun_out/hwq/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value'],2), d['ms_per_step'])"; done
