#!/bin/bash
# hh_ice_balance phase times (create / filters / sweeps / finalize / free) for the e2e and drop-in matrices
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/icep && export TMPDIR=/tmp
O=gpurun_out/icep
for c in e2e dropin; do HH_BUILD_DEBUG=1 timeout -k 10 300 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu > $O/$c.log 2>&1 || exit 1
  echo "== $c"; grep "^\[ice\]" $O/$c.log | tail -4; done
