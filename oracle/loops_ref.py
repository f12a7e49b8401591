"""CPU oracle for HICCUPS loop calling (test infrastructure only: imported by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg).

Restates HiCHap/StructureFind.py ``CallPeaks`` per-chromosome preparation
(:2003-2032), ``pcaller`` (:1631-1948) and ``lambdachunk`` (:1617-1629)
with a dense band instead of ~w^2 shifted sparse diagonal matrices per
window width:

* the reference's ``sparse.diags(Pool_*[w][(i, j)], Offsets_*[w][(i, j)])``
  is the band shifted by (i - w, j - w): S[r, c] = src[r + i - w, c + j - w],
  zero outside the matrix and outside the source's stored diagonals (raw:
  0..num-1 with the main diagonal removed; balanced and expected: ww..num-1);
* donut (``'K'``): offsets (a, b) in [-w, w]^2 with a != 0, b != 0, not both
  within pw; lower-left (``'Y'``): a in [1, w], b in [-w, -1] minus
  a in [1, pw], b in [-pw, -1]; raw reads over the lower-left region decide
  (>= 16) the window width per pixel, and the widening stops when fewer than
  10 % of the still-pending pixels became valid (:1776-1830);
* expected E = EM * (sum balanced / sum expected) * bias_i * bias_j; Poisson
  p = 1 - cdf_{rv}(O) per lambda chunk (rv = the chunk's upper edge, strict
  (lv, rv) membership), BH within each chunk (statsmodels fdr_bh restated:
  statsmodels is absent), q <= 0.05, gap filter +-5 bins, donut AND
  lower-left (:1843-1948).

Pinned by tests/golden/loops_*.npz (tests/golden/make_golden_loops.py runs the
reference's own ``pcaller``).
"""
from __future__ import annotations

import numpy as np


def peaks_parameter(res):
    """Peaks_Parameter (:1596-1615): (pw, ww, maxww, maxapart, sig)."""
    if res >= 20000:
        pw, ww = 1, 3
    elif res >= 10000:
        pw, ww = 2, 5
    else:
        pw, ww = 4, 7
    return pw, ww, 20, 2000000, 0.05


def biases_from_weights(weights):
    """CallPeaks :2007-2010: 1 / weight; weight == 0 -> 0; NaN stays NaN."""
    tmp = np.asarray(weights, dtype=np.float64)
    mask = np.logical_not(tmp == 0) | np.isnan(tmp)
    biases = np.zeros_like(tmp)
    biases[mask] = 1 / tmp[mask]
    return biases


def prepare(H_raw, weights, res, allelic=False):
    """Dense bands + isotonic expected (:2003-2032).  Returns a dict."""
    from sklearn import isotonic
    pw, ww, maxww, maxapart, sig = peaks_parameter(res)
    H = np.asarray(H_raw)
    N = H.shape[0]
    if not allelic:
        w = np.asarray(weights, dtype=np.float64)
        cH = np.nan_to_num(H.astype(float) * w[:, None] * w[None, :])
        biases = biases_from_weights(w)
    else:
        cH = H.astype(float)
        biases = np.ones(N)
    num = maxapart // res + maxww + 1
    r = np.arange(N)[:, None]
    d = np.arange(num)[None, :]
    inside = (r + d) < N
    cc = np.minimum(r + d, N - 1)
    Hb = np.where(inside, H[r, cc], 0).astype(np.float64)
    Hb[:, 0] = 0                                  # H - diag(H) (:2018)
    Cb = np.where(inside & (d >= ww), cH[r, cc], 0.0)
    x = np.arange(ww, num)
    y = [np.diagonal(cH, i).mean() for i in x]
    IR = isotonic.IsotonicRegression(increasing="auto")
    IR.fit(x, y)
    predictE = IR.predict(x)
    predictE[predictE < 0] = 0
    Eall = np.zeros(num)
    Eall[ww:] = predictE
    Eb = np.where(inside, Eall[None, :] * np.ones((N, 1)), 0.0)
    return dict(N=N, num=num, pw=pw, ww=ww, maxww=maxww, maxapart=maxapart, sig=sig, res=res,
                Hb=Hb, Cb=Cb, Eb=Eb, Eall=Eall, biases=biases, allelic=allelic)


def _src(B, R, C):
    """Band value at (R, C) (0 outside the matrix / stored diagonals)."""
    N, num = B.shape
    D = C - R
    ok = (R >= 0) & (R < N) & (D >= 0) & (D < num)
    out = np.zeros(R.shape)
    out[ok] = B[R[ok], D[ok]]
    return out


def region_sum(B, xi, yi, offsets):
    s = np.zeros(xi.shape)
    for a, b in offsets:
        s += _src(B, xi + a, yi + b)
    return s


def donut_offsets(w, pw):
    return [(a, b) for a in range(-w, w + 1) for b in range(-w, w + 1)
            if a != 0 and b != 0 and not (abs(a) <= pw and abs(b) <= pw)]


def lowerleft_offsets(w, pw):
    return [(a, b) for a in range(1, w + 1) for b in range(-w, 0) if not (a <= pw and b >= -pw)]


def candidates(P, gap=None):
    """M.nonzero() restricted to ww <= d <= maxapart // res (:1727-1730), plus
    the allelic gap / blanking filter (:1731-1759)."""
    Hb, ww = P["Hb"], P["ww"]
    N, num = Hb.shape
    rr, dd = np.nonzero(Hb)
    o = np.lexsort((dd, rr))
    xi, yi = rr[o], rr[o] + dd[o]
    m = ((yi - xi) >= ww) & ((yi - xi) <= (P["maxapart"] // P["res"]))
    xi, yi = xi[m], yi[m]
    if P["allelic"]:
        gs = set(int(g) for g in (gap if gap is not None else []))
        keep = np.ones(xi.size, dtype=bool)

        def Hval(R, C):  # M.toarray()[R][C]: NumPy wraps index -1, IndexError -> 1
            if C >= N or R >= N:
                return 1
            return _src(Hb, np.array([R % N]), np.array([C % N]))[0]
        for k in range(xi.size):
            x, y = int(xi[k]), int(yi[k])
            if x in gs and y in gs:
                keep[k] = False
            left = Hval(x - 1, y)
            top = Hval(x, y + 1)
            bottom = Hval(x, y - 1)
            if left * left * top * bottom == 0:   # left and right are the same cell (:1747-1754)
                keep[k] = False
        xi, yi = xi[keep], yi[keep]
    return xi, yi


def neighbourhood(P, xi, yi):
    """The window-widening loop (:1776-1830): per pixel the K / Y sums of the
    balanced and expected bands at its first width with >= 16 lower-left raw
    reads; `valid` False for pixels that never got one."""
    pw, ww, maxww = P["pw"], P["ww"], P["maxww"]
    n = xi.size
    S = {fl: np.zeros(n) for fl in "KY"}
    E = {fl: np.zeros(n) for fl in "KY"}
    pending = np.arange(n)
    ini = n
    widths = []
    for w in range(ww, maxww + 1):
        px, py = xi[pending], yi[pending]
        reads = region_sum(P["Hb"], px, py, lowerleft_offsets(w, pw))
        ok = reads >= 16
        idx = pending[ok]
        ko, yo = donut_offsets(w, pw), lowerleft_offsets(w, pw)
        S["K"][idx] = region_sum(P["Cb"], xi[idx], yi[idx], ko)
        E["K"][idx] = region_sum(P["Eb"], xi[idx], yi[idx], ko)
        S["Y"][idx] = region_sum(P["Cb"], xi[idx], yi[idx], yo)
        E["Y"][idx] = region_sum(P["Eb"], xi[idx], yi[idx], yo)
        ratio = idx.size / float(ini)
        pending = pending[~ok]
        ini = pending.size
        widths.append((w, int(idx.size), ratio))
        if ratio < 0.1:
            break
    valid = np.ones(n, dtype=bool)
    valid[pending] = False
    return S, E, valid, widths


def lambdachunk(E):
    """lambdachunk (:1617-1629)."""
    numbin = int(np.ceil(np.log(E.max()) / np.log(2) * 3 + 1))
    pool = []
    for i in range(1, numbin + 1):
        if i == 1:
            lv, rv = 0, 1
        else:
            lv = np.power(2, ((i - 2) / 3.))
            rv = np.power(2, ((i - 1) / 3.))
        idx = np.where((E > lv) & (E < rv))[0]
        pool.append((lv, rv, idx))
    return pool


def fdr_bh(p):
    """statsmodels fdrcorrection (method 'indep'): corrected p-values."""
    p = np.asarray(p)
    o = np.argsort(p)
    ps = p[o]
    n = len(ps)
    ecdf = np.arange(1, n + 1) / float(n)
    corr = np.minimum.accumulate((ps / ecdf)[::-1])[::-1]
    corr[corr > 1] = 1
    out = np.empty_like(corr)
    out[o] = corr
    return out


def significance(P, xi, yi, S, E, valid):
    """:1832-1948 -> {(x*res, y*res): (O, fold, p, q)} for donut and lower-left."""
    from scipy.stats import poisson
    N, res, sig, ww = P["N"], P["res"], P["sig"], P["ww"]
    mask = (E["K"] != 0) & (E["Y"] != 0) & valid
    xi, yi = xi[mask], yi[mask]
    gaps = np.nonzero(P["Hb"].sum(axis=1) == 0)[0]   # rows of the band matrix M with no contact
    gapset = set(int(g) for g in gaps)
    out = {}
    for fl in "KY":
        ratio = S[fl][mask] / E[fl][mask]
        e_base = P["Eall"][yi - xi]
        cem = e_base * ratio
        nz = cem != 0
        x, y, cem = xi[nz], yi[nz], cem[nz]
        Ev = cem * P["biases"][x] * P["biases"][y]
        m = Ev > 0
        Ev, x, y = Ev[m], x[m], y[m]
        Ov = P["Hb"][x, y - x]
        fold = Ov / Ev
        pv = np.ones(x.size)
        qv = np.ones(x.size)
        for lv, rv, idx in (lambdachunk(Ev) if Ev.size else []):
            if idx.size > 0:
                cp = 1 - poisson(rv).cdf(Ov[idx])
                pv[idx] = cp
                qv[idx] = fdr_bh(cp)
        rej = qv <= sig
        x, y, Ov, Ev, fold, pv, qv = x[rej], y[rej], Ov[rej], Ev[rej], fold[rej], pv[rej], qv[rej]
        if gapset:
            keep = []
            for i in range(x.size):
                lo = (x[i] - 5) if (x[i] > 5) else 0
                up = (x[i] + 5) if ((x[i] + 5) < N) else (N - 1)
                r1 = set(range(lo, up))
                lo = (y[i] - 5) if (y[i] > 5) else 0
                up = (y[i] + 5) if ((y[i] + 5) < N) else (N - 1)
                if not ((r1 | set(range(lo, up))) & gapset):
                    keep.append(i)
            keep = np.array(keep, dtype=np.int64)
            x, y, Ov, fold, pv, qv = x[keep], y[keep], Ov[keep], fold[keep], pv[keep], qv[keep]
        out[fl] = {(int(a) * res, int(b) * res): (o, f, p_, q_) for a, b, o, f, p_, q_ in zip(x, y, Ov, fold, pv, qv)}
    common = set(out["K"]) & set(out["Y"])
    return {k: out["K"][k] for k in common}, {k: out["Y"][k] for k in common}


def pcaller(H_raw, weights, res, allelic=False, gap=None):
    """One chromosome of CallPeaks: (Donuts, LL) as the reference returns them."""
    P = prepare(H_raw, weights, res, allelic)
    xi, yi = candidates(P, gap)
    S, E, valid, _ = neighbourhood(P, xi, yi)
    return significance(P, xi, yi, S, E, valid)
