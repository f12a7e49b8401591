#!/bin/bash
# C5 line under Krylov block counts per cycle (hh_tune pca_p)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
for p in "$@"; do
  HH_PCA_P=$p timeout -k 10 300 python -u bench.py --config c5 --no-cpu > $O/c5_p$p.log 2>&1 || exit 1
  echo "P=$p $(tail -1 $O/c5_p$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value'],1), d['config']['serial_step_ms'], [(k['kernel'][:8], round(k['total_ms'],1)) for k in [r]+r['other_kernels']], sum(d['config']['pca_products_per_chrom'].values()), d['config']['pca_all_converged'])")"
done
