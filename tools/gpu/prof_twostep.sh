#!/bin/bash
# TwoStep lines' PMC traffic at the current build (FETCH_SIZE and WRITE_SIZE in
# separate passes, summarised by tools/pmc_summary.py with the sources'
# fingerprint and workload in _meta, which bench.py then reports as
# roofline.traffic).  tools/gpu/prof_twostep.sh outdir tag commit
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; TAG=${2:-r6}; COMMIT=${3:-unknown}; mkdir -p $O
for c in twostep twostep_genome; do
  timeout -k 10 300 python3 -u bench.py --config $c --no-cpu > $O/${c}_bench.log 2>&1 || exit 1
  cd /tmp
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d /tmp/pts${c}f -o f --output-format csv -- python3 $R/bench.py --config $c --no-cpu --main-only --steps 3 --warmup 1 > $O/${c}_pmc_f.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d /tmp/pts${c}w -o w --output-format csv -- python3 $R/bench.py --config $c --no-cpu --main-only --steps 3 --warmup 1 > $O/${c}_pmc_w.log 2>&1 || exit 1
  python3 $R/tools/pmc_summary.py $(find /tmp/pts${c}f -name "*counter_collection.csv" | head -1) $(find /tmp/pts${c}w -name "*counter_collection.csv" | head -1) $O/${TAG}_${c}_pmc.json "$COMMIT" - $c $O/${c}_bench.log > $O/${c}_pmc_summary.log 2>&1 || exit 1
  cd $R
done
