set -o pipefail
mkdir -p gpurun_out
HH_DEVICE=0 HH_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --nnz 1e9 \
  --steps 10 --warmup 2 > gpurun_out/r1v8_c4_2rank_gloo_bench.log 2>&1
