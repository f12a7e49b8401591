set -o pipefail
mkdir -p gpurun_out
HH_TUNE=band_concurrent=1,split_tiles=0 timeout -k 10 200 python -u tools/probe_shards.py 8 0 > gpurun_out/shards_split0.log 2>&1 && \
HH_TUNE=band_concurrent=1,split_tiles=1 timeout -k 10 200 python -u tools/probe_shards.py 8 0 > gpurun_out/shards_split1.log 2>&1 && \
timeout -k 10 300 python -u tools/probe_knobs.py "band_concurrent=0,split_tiles=0" "band_concurrent=1,split_tiles=1" > gpurun_out/knobs_split.log 2>&1
