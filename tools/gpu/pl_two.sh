# path checks: pairs and loops configs with 2 ranks sharing cuda:0
set -o pipefail
mkdir -p gpurun_out
HH_DEVICE=0 HH_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29536 bench.py --gpus 2 --config pairs \
  --pairs 2e7 --steps 2 --warmup 1 > gpurun_out/r1v8_pairs_2rank_gloo.log 2>&1 && \
HH_DEVICE=0 HH_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29537 bench.py --gpus 2 --config loops \
  --steps 2 --warmup 1 > gpurun_out/r1v8_loops_2rank_gloo.log 2>&1
