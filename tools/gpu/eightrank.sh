# path check of the N=8 driver on one GPU (8 ranks share cuda:0, gloo exchange);
# timings are meaningless (all ranks contend for one device)
set -o pipefail
mkdir -p gpurun_out
HH_DEVICE=0 HH_DIST_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 \
  --steps 5 --warmup 1 > gpurun_out/r1v8_c4_8rank_gloo_bench.log 2>&1
