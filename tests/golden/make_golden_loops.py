#!/usr/bin/env python3
"""Golden vectors for HICCUPS loop calling from the REFERENCE's own code.

Run in the build container only (reads /root/reference, absent on the GPU box):

    python tests/golden/make_golden_loops.py

As in make_golden.py, the Python-2 source TEXT of HiCHap/StructureFind.py is
converted with lib2to3 in memory and the methods ``Peaks_Parameter``,
``lambdachunk`` and ``pcaller`` are executed.  ``CallPeaks`` (:1971-2043)
reads cooler files; its per-chromosome preparation (raw / balanced dense
matrices, biases, band diagonals, isotonic expected) is restated below line
by line from :2003-2032 (cooler is absent).  statsmodels is absent too:
``multipletests(..., method='fdr_bh')`` is injected as a restatement of
statsmodels' ``fdrcorrection`` (argsort, p / (rank / n), reversed running
minimum, capped at 1).  scipy.stats.poisson and sklearn.isotonic are the
real libraries.  Nothing converted is written to disk.
"""
from __future__ import annotations

import ast
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/HiCHap"
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

from make_golden import _py3_source  # noqa: E402

METHODS = ["Peaks_Parameter", "lambdachunk", "pcaller"]


def multipletests(pvals, alpha=0.05, method="fdr_bh"):
    """statsmodels.sandbox.stats.multicomp.multipletests, method 'fdr_bh'."""
    assert method == "fdr_bh"
    pvals = np.asarray(pvals)
    sortind = np.argsort(pvals)
    ps = np.take(pvals, sortind)
    nobs = len(ps)
    ecdf = np.arange(1, nobs + 1) / float(nobs)
    reject = ps <= ecdf * alpha
    if reject.any():
        reject[:max(np.nonzero(reject)[0])] = True
    raw = ps / ecdf
    corr = np.minimum.accumulate(raw[::-1])[::-1]
    corr[corr > 1] = 1
    out_r = np.empty_like(reject)
    out_r[sortind] = reject
    out_p = np.empty_like(corr)
    out_p[sortind] = corr
    return out_r, out_p, None, None


def load_reference():
    from scipy import sparse
    from scipy.stats import poisson
    from sklearn import isotonic
    for name, val in (("int", int), ("float", float), ("bool", bool)):
        if not hasattr(np, name):
            setattr(np, name, val)
    ns = {"np": np, "sparse": sparse, "poisson": poisson, "multipletests": multipletests,
          "isotonic": isotonic, "xrange": range}
    tree = ast.parse(_py3_source(os.path.join(REF, "StructureFind.py")))
    cls = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "StructureFind"][0]
    meths = [n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name in METHODS]
    assert {m.name for m in meths} == set(METHODS)
    klass = ast.ClassDef(name="RefSF", bases=[], keywords=[], body=meths, decorator_list=[])
    exec(compile(ast.fix_missing_locations(ast.Module(body=[klass], type_ignores=[])), "<StructureFind>", "exec"),
         ns)
    return ns


def synth_chrom(rng, N, n_loops=14, A=60.0):
    """Raw symmetric int counts: power-law decay + planted loop pixels."""
    i = np.arange(N)
    d = np.abs(i[:, None] - i[None, :])
    vis = rng.lognormal(0, 0.25, N)
    lam = A * (d + 1.0) ** -1.0 * vis[:, None] * vis[None, :]
    loops = []
    for _ in range(n_loops):
        a = int(rng.integers(10, N - 60))
        b = a + int(rng.integers(8, 45))
        loops.append((a, b))
        for da in (-1, 0, 1):
            for db in (-1, 0, 1):
                f = 8.0 if (da, db) == (0, 0) else 3.0
                lam[a + da, b + db] *= f
                lam[b + db, a + da] *= f
    H = rng.poisson(np.triu(lam))
    H = np.triu(H) + np.triu(H, 1).T
    gaps = rng.choice(N, size=max(2, N // 60), replace=False)
    H[gaps, :] = 0
    H[:, gaps] = 0
    return H.astype(np.int64), np.array(sorted(loops)), np.sort(gaps)


def ice_weights(H):
    """Simple cis ICE (matrix balancing) for the synthetic weights; masked
    rows -> NaN (cooler semantics: weight NaN where the bin is filtered)."""
    A = H.astype(float).copy()
    np.fill_diagonal(A, 0)
    b = np.ones(A.shape[0])
    keep = A.sum(1) > 0
    b[~keep] = 0
    for _ in range(200):
        m = (A * b[:, None] * b[None, :]).sum(1)
        nz = m[m != 0]
        m = m / nz.mean()
        m[m == 0] = 1
        b /= m
    w = b.copy()
    w[w == 0] = np.nan
    return w


def prepare(sf, H_raw, weights, res, allelic=False):
    """CallPeaks' per-chromosome preparation (:2003-2032)."""
    from scipy import sparse
    from sklearn import isotonic
    H = H_raw.copy()
    if not allelic:
        cH = H.astype(float) * weights[:, None] * weights[None, :]
        cH = np.nan_to_num(cH)
        tmp = weights
        mask = np.logical_not((tmp == 0)) | np.isnan(tmp)
        biases = np.zeros_like(tmp)
        biases[mask] = 1 / tmp[mask]
    else:
        cH = H.copy()
        biases = np.ones(H.shape[0], )
    H = H - np.diag(H.diagonal())
    chromLen = H.shape[0]
    num = sf.maxapart // sf.Res + sf.maxww + 1
    Diags = [np.diagonal(H, i) for i in np.arange(num)]
    M = sparse.diags(Diags, np.arange(num), format="csr")
    x = np.arange(sf.ww, num)
    y = []
    cDiags = []
    for i in x:
        diag = np.diagonal(cH, i)
        y.append(diag.mean())
        cDiags.append(diag)
    cM = sparse.diags(cDiags, x, format="csr")
    IR = isotonic.IsotonicRegression(increasing="auto")
    IR.fit(x, y)
    return dict(M=M, cM=cM, biases=biases, IR=IR, chromLen=chromLen, Diags=Diags, cDiags=cDiags, num=num)


def flat(calls):
    keys = sorted(calls)
    pos = np.array(keys, dtype=np.int64).reshape(-1, 2)
    vals = np.array([calls[k] for k in keys], dtype=np.float64).reshape(-1, 4)
    return pos, vals


def main():
    ref = load_reference()
    rng = np.random.default_rng(20201017)
    cases = {}
    for name, N, res, allelic in (("loops_trad_n360", 360, 40000, False),
                                  ("loops_allelic_n300", 300, 40000, True)):
        H, loops, gaps = synth_chrom(rng, N)
        w = ice_weights(H)
        sf = ref["RefSF"]()
        sf.Res = res
        sf.Peaks_Parameter()
        prep = prepare(sf, H, w, res, allelic)
        gap_list = list(gaps) if allelic else None
        Donuts, LL = sf.pcaller(Allelic=allelic if allelic else False, Gap=gap_list, **prep)
        pd, vd = flat(Donuts)
        pl, vl = flat(LL)
        assert np.array_equal(pd, pl)
        cases[name] = dict(H=H, weights=w, res=np.int64(res), allelic=np.int64(allelic), gaps=gaps,
                           planted=loops, pos=pd, donut=vd, ll=vl)
        print(name, "calls:", len(pd), "planted:", len(loops))
    for name, d in cases.items():
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **d)
        print("wrote", path)


if __name__ == "__main__":
    main()
