# path check: C5 (per-chromosome LPT over ranks) with 2 ranks sharing cuda:0
set -o pipefail
mkdir -p gpurun_out
HH_DEVICE=0 HH_DIST_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --config c5 \
  --steps 2 --warmup 1 > gpurun_out/r1v8_c5_2rank_gloo.log 2>&1
