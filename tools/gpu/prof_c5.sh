#!/bin/bash
# C5 evidence at the current build: the bench line and the PMC traffic of its
# kernels (FETCH_SIZE and WRITE_SIZE in separate passes), summarised with the
# source fingerprint and workload.   tools/gpu/prof_c5.sh outdir tag commit
cd "${GRAFT_REPO_ROOT:-/root/repo}" && R=$PWD && export TMPDIR=/tmp
O=$R/gpurun_out/$1; TAG=${2:-r5}; COMMIT=${3:-unknown}; mkdir -p $O
timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu > $O/c5_bench.log 2>&1 || exit 1
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d /tmp/pc5f -o f --output-format csv -- python3 $R/bench.py --config c5 --no-cpu --steps 2 --warmup 0 > $O/c5_pmc_f.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d /tmp/pc5w -o w --output-format csv -- python3 $R/bench.py --config c5 --no-cpu --steps 2 --warmup 0 > $O/c5_pmc_w.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py $(find /tmp/pc5f -name "*counter_collection.csv" | head -1) $(find /tmp/pc5w -name "*counter_collection.csv" | head -1) $O/${TAG}_c5_pmc.json "$COMMIT" - c5 $O/c5_bench.log > $O/c5_pmc_summary.log 2>&1 || exit 1
python3 - $O/${TAG}_c5_pmc.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if k != "_meta" and any(s in k for s in ("k_ortho", "k_cor_sym", "k_syrk")):
        print(k[:50], round(v["traffic_bytes"] / 1e6, 3), "MB/dispatch", v["dispatches"])
PY
