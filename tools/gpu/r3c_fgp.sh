#!/bin/bash
# flat column-group size: FETCH_SIZE of the flat kernel at the automatic 44 vs 88 tiles per group
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3c && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3c
R=$GRAFT_REPO_ROOT
cd /tmp
for g in 0 88; do
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d /tmp/fg$g -o f --output-format csv -- python3 $R/tools/probe_knobs.py --iters 4 "flat_group=$g" > $O/fgp_$g.log 2>&1 || exit 1
python3 $R/tools/pmc_counters.py $(find /tmp/fg$g -name "*counter_collection.csv" | head -1) $O/fgp_$g.json k_sweep_flatw > /dev/null 2>&1 || exit 1
python3 -c "import json; d=json.load(open('$O/fgp_$g.json')); [print('$g', k[:40], v['FETCH_SIZE']) for k,v in d.items()]"
done
