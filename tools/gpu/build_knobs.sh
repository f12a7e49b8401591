#!/bin/bash
# Sweep times of one bench config under several BUILD-time knobs (one matrix
# build each, tools/probe_knobs.py --build), the run-time setting fixed.
#   tools/gpu/build_knobs.sh outdir config "run k=v,..." "build k=v,..." ...   (config "" = C4)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
O=gpurun_out/$1; C=$2; RUN=$3; shift 3; mkdir -p $O
i=0
for b in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python3 -u tools/probe_knobs.py ${C:+--config $C} --build "$b" --iters 20 "$RUN" > $O/${C:-c4}_$i.log 2>&1 || { echo "$b failed"; tail -3 $O/${C:-c4}_$i.log; exit 1; }
  echo "[${C:-c4} build $b] $(grep -v amdgpu $O/${C:-c4}_$i.log | grep -E 'build|sweep' | tr '\n' ' ' | cut -c1-400)"
done
