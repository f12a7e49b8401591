#!/usr/bin/env python3
"""Generate golden vectors from the REFERENCE's own functions.

Run in the build container only (it reads /root/reference, which does not
exist on the GPU box):

    python tests/golden/make_golden.py

How the reference is executed: the Python-2 source TEXT of
``HiCHap/matrixBuilding.py`` and ``HiCHap/StructureFind.py`` is converted with
``lib2to3`` in memory, the needed function / method definitions are extracted
with ``ast`` and executed with the removed NumPy aliases shimmed
(``np.int/np.float/np.bool``).  Nothing converted is written to disk; only the
inputs and outputs (data) are saved as ``.npz`` fixtures next to this script.

Deviation: ``PCA`` is injected as ``sklearn PCA(svd_solver='full')`` because the
reference's default is randomized above 500×500.
"""
from __future__ import annotations

import ast
import os
import sys
import warnings
from collections import OrderedDict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/HiCHap"
sys.path.insert(0, REPO)

from hichap_master_amd import synth  # noqa: E402

MB_FUNCS = [
    "Sort_Chromosomes", "Gap_definedLowRes", "Non_Gap_DefinedLowRes", "Trans2symmetryLowRes",
    "Correct_VC", "GenomeWideMatrixCorrection", "Coverage_M", "Gap_defined", "Non_Gap_Defined",
    "Trans2symmetry", "TwoStepCorrection", "IntraChromMatrixCorrection",
]
SF_METHODS = [
    "Distance_Decay", "Get_PCA", "Select_PC_new", "Select_Allelic_PC", "Get_Gap", "Gap_Filter",
    "Get_DI", "Sliding_Approach",
]


def _py3_source(path):
    warnings.simplefilter("ignore")
    from lib2to3 import refactor
    text = open(path).read()
    if not text.endswith("\n"):
        text += "\n"
    tool = refactor.RefactoringTool(refactor.get_fixers_from_package("lib2to3.fixes"))
    return str(tool.refactor_string(text, os.path.basename(path)))


def _namespace():
    from scipy import sparse
    from sklearn.decomposition import PCA as _PCA
    import math

    for name, val in (("int", int), ("float", float), ("bool", bool)):
        if not hasattr(np, name):
            setattr(np, name, val)

    def PCA(n_components=3):  # exact SVD, see module docstring
        return _PCA(n_components=n_components, svd_solver="full")

    return {"np": np, "math": math, "sparse": sparse, "PCA": PCA,
            "OrderedDict": OrderedDict, "xrange": range}


def load_reference():
    ns = _namespace()
    tree = ast.parse(_py3_source(os.path.join(REF, "matrixBuilding.py")))
    fdefs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in MB_FUNCS]
    assert {f.name for f in fdefs} == set(MB_FUNCS)
    exec(compile(ast.Module(body=fdefs, type_ignores=[]), "<matrixBuilding>", "exec"), ns)

    tree = ast.parse(_py3_source(os.path.join(REF, "StructureFind.py")))
    cls = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "StructureFind"][0]
    meths = [n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name in SF_METHODS]
    assert {m.name for m in meths} == set(SF_METHODS)
    klass = ast.ClassDef(name="RefSF", bases=[], keywords=[], body=meths, decorator_list=[])
    exec(compile(ast.fix_missing_locations(ast.Module(body=[klass], type_ignores=[])),
                 "<StructureFind>", "exec"), ns)
    return ns


def gen_twostep(ref, rng, N, drop_rows, no_gap_m=False):
    TM = synth.dense_chrom(N, rng, A=60.0)
    MM, PM = synth.haplotype_pair(TM, rng, drop_rows=drop_rows)
    if no_gap_m:
        MM = MM + 1  # every row fully covered -> Gap_M empty -> SUM branch
    nmm, npm, gm, gp = ref["TwoStepCorrection"](TM, MM, PM)
    return dict(TM=TM, MM=MM, PM=PM, Nor_MM=nmm, Nor_PM=npm,
                Gap_M=np.asarray(gm, dtype=np.int64), Gap_P=np.asarray(gp, dtype=np.int64))


def gen_genomewide(ref, rng, sizes):
    names = [str(i + 1) for i in range(len(sizes) - 1)] + ["X"]
    n = sum(sizes)
    T_M = np.zeros((n, n), dtype=np.int64)
    H_M = np.zeros((2 * n, 2 * n), dtype=np.int64)
    bins, hbins = {}, {}
    s = 0
    for nm, L in zip(names, sizes):
        bins[nm] = (s, s + L - 1)
        s += L
    for k, (nm, L) in enumerate(zip(names, sizes)):
        hbins["M" + nm] = (bins[nm][0], bins[nm][1])
        hbins["P" + nm] = (n + bins[nm][0], n + bins[nm][1])
    for nm, L in zip(names, sizes):
        a, b = bins[nm]
        T = synth.dense_chrom(L, rng, A=40.0)
        T_M[a:b + 1, a:b + 1] = T
        Mx, Px = synth.haplotype_pair(T, rng)
        ma, mb = hbins["M" + nm]
        pa, pb = hbins["P" + nm]
        H_M[ma:mb + 1, ma:mb + 1] = Mx
        H_M[pa:pb + 1, pa:pb + 1] = Px
    # sparse trans + M/P cross contacts
    for X in (T_M, H_M):
        m = X.shape[0]
        noise = rng.binomial(1, 0.03, size=(m, m)) * rng.integers(1, 3, size=(m, m))
        noise = np.triu(noise, 1)
        X += noise + noise.T
    Nor = ref["GenomeWideMatrixCorrection"](bins, hbins, T_M, H_M)
    return dict(T_M=T_M, H_M=H_M, names=np.array(names), sizes=np.array(sizes, dtype=np.int64),
                Nor=Nor)


def gen_compartment(ref, rng, N):
    M = synth.dense_chrom(N, rng, A=80.0, comp_len=(8, 30)).astype(np.float64)
    sf = ref["RefSF"]()
    sf.Res = 100000
    dec, G, NG = sf.Distance_Decay(M=M.copy(), G_array=None)
    dec0 = dec.copy()
    pca, Cor, OE = sf.Get_PCA(distance_bin=dec.copy(), M=M, NG_array=NG, SA=False)
    pc = sf.Select_PC_new(Cor, OE[NG], pca)
    full = np.zeros(N)
    full[NG] = pc
    # haplotype selection against the traditional PC
    raw = []
    for i in range(len(pca)):
        t = np.zeros(N)
        t[NG] = pca[i]
        raw.append(t)
    raw = np.array(raw)
    trad = full + rng.normal(0, 0.01, size=N)
    allelic = sf.Select_Allelic_PC(raw, trad)
    return dict(M=M, decline=dec0, G=np.asarray(G, np.int64), NG=np.asarray(NG, np.int64),
                pcs=np.asarray(pca), Cor=Cor, OE=OE, pc=full, trad=trad, allelic=allelic)


def gen_compartment_sa(ref, rng, N, res):
    """Get_PCA(SA=True): the Sliding_Approach O/E (StructureFind.py:274-299,
    window 600 kb -> step = 600000 // res // 2) feeding corrcoef + PCA(3) +
    Select_PC_new."""
    M = synth.dense_chrom(N, rng, A=60.0, comp_len=(8, 30)).astype(np.float64)
    sf = ref["RefSF"]()
    sf.Res = res
    dec, G, NG = sf.Distance_Decay(M=M.copy(), G_array=None)
    dec0 = dec.copy()
    pca, Cor, OE = sf.Get_PCA(distance_bin=dec.copy(), M=M, NG_array=NG, SA=True)
    pc = sf.Select_PC_new(Cor, OE[NG], pca)
    full = np.zeros(N)
    full[NG] = pc
    return dict(M=M, res=np.int64(res), decline=dec0, NG=np.asarray(NG, np.int64), pcs=np.asarray(pca),
                Cor=Cor, OE=OE, pc=full)


def gen_di(ref, rng, N, test_type, res=40000, min_tad=200000, window=600000):
    M = synth.dense_chrom(N, rng, A=30.0, gap_frac=0.04).astype(np.float64)
    # balanced-like float matrix with NaN->0 as Data_preprocess does
    w = 1.0 / np.sqrt(np.maximum(M.sum(axis=1), 1.0))
    Mb = M * w[:, None] * w[None, :]
    sf = ref["RefSF"]()
    sf.Res = res
    sf.minTAD = min_tad
    sf.window = window
    sf.test_type = test_type
    gap = list(sf.Get_Gap(Mb))
    if 0 not in gap:
        gap.insert(0, 0)
    if N - 1 not in gap:
        gap.append(N - 1)
    gap = np.array(gap)
    wb = int(window / res)
    DI = sf.Get_DI(Mb, gap, np.ones(N, dtype=int) * wb)
    filt = sf.Gap_Filter(gap, Mb)
    return dict(M=Mb, gap=np.asarray(gap, np.int64), DI=DI, window_bins=np.int64(wb),
                lb=np.int64(int(min_tad / res)), gap_filtered=np.asarray(filt, np.int64))


def main_sa():
    """Only the Sliding_Approach cases (own seed: the other fixtures keep
    their bytes)."""
    ref = load_reference()
    rng = np.random.default_rng(20201020)
    out = {"compartment_sa_n120": gen_compartment_sa(ref, rng, 120, 100000),
           "compartment_sa_n150": gen_compartment_sa(ref, rng, 150, 50000)}
    for name, d in out.items():
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **d)
        print("wrote", path, {k: np.shape(v) for k, v in d.items()})


def main():
    ref = load_reference()
    out = {}
    rng = np.random.default_rng(20201015)
    out["twostep_gaps_n96"] = gen_twostep(ref, rng, 96, drop_rows=6)
    out["twostep_gaps_n160"] = gen_twostep(ref, rng, 160, drop_rows=12)
    out["twostep_nogapM_n80"] = gen_twostep(ref, rng, 80, drop_rows=0, no_gap_m=True)
    out["genomewide_3chrom"] = gen_genomewide(ref, rng, [40, 28, 20])
    out["compartment_n150"] = gen_compartment(ref, rng, 150)
    out["compartment_n260"] = gen_compartment(ref, rng, 260)
    out["di_ttest_n220"] = gen_di(ref, rng, 220, "ttest")
    out["di_chitest_n220"] = gen_di(ref, rng, 220, "chitest")
    for name, d in out.items():
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **d)
        print("wrote", path, {k: np.shape(v) for k, v in d.items()})


if __name__ == "__main__":
    import sys
    main_sa() if sys.argv[1:] == ["sa"] else main()
