# Other BASELINE configs at N=1 plus a 2-rank path check of the sharded
# driver on the one GPU of the box (both ranks on cuda:0, gloo exchange;
# the N>1 RCCL runs are the driver's, on an 8-GPU node).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config c3 > gpurun_out/r1v8_c3_bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c2 --steps 200 > gpurun_out/r1v8_c2_bench.log 2>&1 && \
HH_DEVICE=0 HH_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --nnz 1e9 \
  --steps 10 --warmup 2 > gpurun_out/r1v8_c4_2rank_gloo_bench.log 2>&1
