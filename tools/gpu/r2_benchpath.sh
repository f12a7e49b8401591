#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2_c4_bench.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --sharded --steps 10 --warmup 2 --no-cpu > gpurun_out/r2_c4_sharded1.log 2>&1 || exit 1
HH_DEVICE=0 HH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --nnz 5e8 > gpurun_out/r2_c4_2rank_gloo.log 2>&1
