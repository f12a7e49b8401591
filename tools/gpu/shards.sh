set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe_shards.py 2,4 0 > gpurun_out/probe_shards24.log 2>&1 && \
HH_TUNE=band_concurrent=1 timeout -k 10 300 python -u tools/probe_shards.py 2,4 0 > gpurun_out/probe_shards24_conc.log 2>&1
