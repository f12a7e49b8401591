set -o pipefail
mkdir -p gpurun_out /tmp/pf /tmp/pw
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d /tmp/pf -o f --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/pmc_f.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d /tmp/pw -o w --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/pmc_w.log 2>&1 && \
python3 tools/pmc_summary.py $(find /tmp/pf -name "*counter_collection.csv" | head -1) $(find /tmp/pw -name "*counter_collection.csv" | head -1) gpurun_out/r1v8_c4_pmc.json > gpurun_out/pmc_summary.log 2>&1
