set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/c5prof -o c5 --output-format csv -- python3 bench.py --config c5 --no-cpu --steps 2 --warmup 1 > gpurun_out/c5_prof.log 2>&1 && \
cp $(find /tmp/c5prof -name "c5_kernel_stats.csv" | head -1) gpurun_out/c5_kernel_stats.csv
