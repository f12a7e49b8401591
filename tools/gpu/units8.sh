set -o pipefail
mkdir -p gpurun_out
HH_TUNE=unit_entries=262144 timeout -k 10 200 python -u tools/probe_shards.py 8 0 > gpurun_out/shards_u256k.log 2>&1 && \
HH_TUNE=unit_entries=524288 timeout -k 10 200 python -u tools/probe_shards.py 8 0 > gpurun_out/shards_u512k.log 2>&1 && \
HH_TUNE=unit_entries=65536 timeout -k 10 200 python -u tools/probe_shards.py 8 0 > gpurun_out/shards_u64k.log 2>&1
