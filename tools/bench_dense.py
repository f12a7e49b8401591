"""Timing of the dense kernels at the configs' sizes (run under rocprofv3
--kernel-trace --stats for per-kernel times).

  compartment: hg19 chr1 at 25 kb (N = 9971), C5's largest chromosome
  two-step:    hg19 chr1 at 40 kb (N = 6232) maternal / paternal
  DI scan:     hg19 chr1 at 10 kb (N = 24926), window 60 bins (C2's TAD scan)
"""
import sys
import time

import numpy as np

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hichap_master_amd import _lib, synth  # noqa: E402
from hichap_master_amd.StructureFind import StructureFind  # noqa: E402
from hichap_master_amd.matrixBuilding import TwoStepCorrection  # noqa: E402

_lib.load()
_lib.require_gpu()
which = sys.argv[1:] or ["comp", "twostep", "di"]
rng = np.random.default_rng(1)


def timed(label, f, *a, **k):
    t0 = time.perf_counter()
    r = f(*a, **k)
    print(f"{label}: {time.perf_counter() - t0:.3f} s (host wall incl. transfers)", flush=True)
    return r


if "comp" in which:
    N = synth.chrom_bins([synth.HG19["1"]], 25000)[0]
    M = synth.dense_chrom(N, rng, A=120.0, comp_len=(40, 200), gap_frac=0.03).astype(np.float64)
    sf = StructureFind(Res=25000)
    for rep in range(2):
        dec, G, NG = timed("Distance_Decay", sf.Distance_Decay, M=M, G_array=None)
        pcs, Cor, OE = timed("Get_PCA", sf.Get_PCA, distance_bin=dec, M=M, NG_array=NG)
        pc = timed("Select_PC_new", sf.Select_PC_new, Cor, OE[NG], pcs)
    n = NG.size
    print(f"compartment N={N} n={n} syrk_flops={float(N) * n * (n + 1):.3e} pca_iters={sf._comp.pca(3)[2]}")

if "twostep" in which:
    N = synth.chrom_bins([synth.HG19["1"]], 40000)[0]
    TM = synth.dense_chrom(N, rng, A=60.0)
    MM, PM = synth.haplotype_pair(TM, rng, drop_rows=50)
    for rep in range(2):
        timed(f"TwoStepCorrection N={N}", TwoStepCorrection, TM, MM, PM)

if "di" in which:
    N = synth.chrom_bins([synth.HG19["1"]], 10000)[0]
    M = np.zeros((N, N))
    band = 200
    for d in range(band):
        v = rng.poisson(30.0 * (d + 1) ** -1.08, size=N - d).astype(float)
        idx = np.arange(N - d)
        M[idx, idx + d] = v
        M[idx + d, idx] = v
    sf = StructureFind(Res=10000)
    sf.TAD_parameter_init(200000, 4000000, 3, 600000, "ttest")
    for rep in range(2):
        timed(f"DI scan N={N}", sf.di_scan, M)
