#!/bin/bash
# C5 bench: concurrent stream count x Krylov cycle length
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for cfg in "4 8" "8 8" "11 8" "8 6" "16 6"; do
  set -- $cfg
  echo "streams=$1 p=$2" >> gpurun_out/r2_c5s.log
  HH_C5_STREAMS=$1 HH_PCA_P=$2 timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu >> gpurun_out/r2_c5s.log 2>&1 || exit 1
done
