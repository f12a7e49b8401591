#!/bin/bash
# gw evidence at the current build: the bench line and the PMC traffic of the
# whole correction (FETCH_SIZE and WRITE_SIZE in separate passes, summarised
# by tools/pmc_summary.py with the source fingerprint and workload in _meta).
#   tools/gpu/prof_gw.sh outdir tag commit
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; TAG=${2:-r5}; COMMIT=${3:-unknown}; mkdir -p $O
timeout -k 10 300 python3 -u bench.py --config gw --no-cpu > $O/gw_bench.log 2>&1 || exit 1
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d /tmp/pgwf -o f --output-format csv -- python3 $R/bench.py --config gw --no-cpu --steps 3 --warmup 0 > $O/gw_pmc_f.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d /tmp/pgww -o w --output-format csv -- python3 $R/bench.py --config gw --no-cpu --steps 3 --warmup 0 > $O/gw_pmc_w.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py $(find /tmp/pgwf -name "*counter_collection.csv" | head -1) $(find /tmp/pgww -name "*counter_collection.csv" | head -1) $O/${TAG}_gw_pmc.json "$COMMIT" - gw $O/gw_bench.log > $O/gw_pmc_summary.log 2>&1 || exit 1
