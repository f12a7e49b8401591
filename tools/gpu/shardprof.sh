set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/shprof -o sh --output-format csv -- python3 tools/probe_shards.py 8 0 > gpurun_out/shardprof.log 2>&1 && \
cp $(find /tmp/shprof -name "sh_kernel_stats.csv" | head -1) gpurun_out/shard8_kernel_stats.csv
