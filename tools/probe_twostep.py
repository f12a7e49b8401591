"""Timing probe of the batched TwoStep (hh_twostep_batch) on the hg19 40 kb
genome (bench.py --config twostep_genome's matrices): ms per genome for each
stream count given on the command line.
    GPU_MAX_HW_QUEUES=8 python tools/probe_twostep.py 1 2 4 8"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hichap_master_amd import _lib, matrixBuilding as mb, synth  # noqa: E402

_lib.load()
_lib.require_gpu()
names = [str(c) for c in range(1, 23)] + ["X"]
Ns = synth.chrom_bins([synth.HG19[c] for c in names], 40000)
gen = torch.Generator(device="cuda").manual_seed(20201025)
rng = np.random.default_rng(20201025)
tra, hap = {}, {}
for c, N in zip(names, Ns):
    tra[c], hap["M" + c], hap["P" + c] = bench._dense_pair_device(int(N), gen, rng, drop_rows=max(1, int(N) // 50))
torch.cuda.synchronize()
print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', '(default)')}", flush=True)
for k in [int(x) for x in sys.argv[1:]]:
    mb.IntraChromMatrixCorrection(tra, hap, n_streams=k)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        mb.IntraChromMatrixCorrection(tra, hap, n_streams=k)
    torch.cuda.synchronize()
    print(f"  n_streams={k}: {(time.perf_counter() - t) / 5 * 1e3:.3f} ms per genome", flush=True)
