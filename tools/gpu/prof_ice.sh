#!/bin/bash
# PMC traffic of an ICE bench line (c4h | c3 | c2 | cis; C4 has prof_c4.sh):
# the line, then FETCH_SIZE and WRITE_SIZE in separate passes, summarised with
# the source fingerprint and workload.   tools/gpu/prof_ice.sh outdir tag commit config
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; TAG=${2:-r5}; COMMIT=${3:-unknown}; CFG=$4; mkdir -p $O
timeout -k 10 300 python3 -u bench.py --config $CFG --no-cpu > $O/${CFG}_bench.log 2>&1 || exit 1
RB=$(python3 -c "import json; print([json.loads(l) for l in open('$O/${CFG}_bench.log') if l.startswith('{\"metric')][-1]['roofline']['real_bytes_per_launch'])")
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d /tmp/pi_${CFG}_f -o f --output-format csv -- python3 $R/bench.py --config $CFG --no-cpu --steps 3 --warmup 1 > $O/${CFG}_pmc_f.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d /tmp/pi_${CFG}_w -o w --output-format csv -- python3 $R/bench.py --config $CFG --no-cpu --steps 3 --warmup 1 > $O/${CFG}_pmc_w.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py $(find /tmp/pi_${CFG}_f -name "*counter_collection.csv" | head -1) $(find /tmp/pi_${CFG}_w -name "*counter_collection.csv" | head -1) $O/${TAG}_${CFG}_pmc.json "$COMMIT" $RB $CFG $O/${CFG}_bench.log > $O/${CFG}_pmc_summary.log 2>&1 || exit 1
head -6 $O/${CFG}_pmc_summary.log | cut -c1-200
