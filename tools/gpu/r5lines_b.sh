#!/bin/bash
# The remaining bench lines and a two-rank path check of the sharded C4 bench
# (both ranks on device 0 over gloo: the N > 1 code path, not RCCL).
#   tools/gpu/r5lines_b.sh outdir
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
bash tools/gpu/lines.sh $1 c5 gw dropin e2e pairs loops || exit 1
for q in 8 16; do  # C5 with more hardware queues (12 stream workers; k_ortho's grid cap follows the env)
GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu > gpurun_out/$1/c5_q$q.log 2>&1 || { tail -5 gpurun_out/$1/c5_q$q.log; exit 1; }
echo "c5 GPU_MAX_HW_QUEUES=$q $(grep '^{"metric"' gpurun_out/$1/c5_q$q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), d['unit'])")"
done
HH_DEVICE=0 HH_DIST_BACKEND=gloo timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/$1/c4_2rank_gloo_pathcheck.log 2>&1 || { tail -20 gpurun_out/$1/c4_2rank_gloo_pathcheck.log; exit 1; }
grep '^{"metric"' gpurun_out/$1/c4_2rank_gloo_pathcheck.log | cut -c1-300
# C5 eigensolver host / device time split per Krylov cycle (diagnostic)
HH_PCA_DEBUG=1 timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu --steps 1 --warmup 0 > gpurun_out/$1/c5_pcadebug.log 2>&1 || { tail -5 gpurun_out/$1/c5_pcadebug.log; exit 1; }
python3 - gpurun_out/$1/c5_pcadebug.log <<'PY'
import re, sys
h = e = g = 0.0; n = 0
for line in open(sys.argv[1]):
    m = re.search(r"host_ms H=([\d.]+) eig=([\d.]+) gpu_wait_ms=([\d.]+)", line)
    if m:
        h += float(m.group(1)); e += float(m.group(2)); g += float(m.group(3)); n += 1
print(f"pca cycles {n}: host H {h:.1f} ms, host eig {e:.1f} ms, gpu wait {g:.1f} ms (summed over all passes)")
PY
