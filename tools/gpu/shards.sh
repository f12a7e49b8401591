set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe_shards.py 8 1 > gpurun_out/probe_shards.log 2>&1 && \
HH_TUNE=band_concurrent=1 timeout -k 10 200 python -u tools/probe_shards.py 8 0 > gpurun_out/probe_shards_conc.log 2>&1
