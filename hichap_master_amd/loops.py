"""HICCUPS loop calling on MI355X — StructureFind.CallPeaks / pcaller
(HiCHap/StructureFind.py:1596-2043).

Per chromosome:

1. host: the raw band (main diagonal removed), the balanced band, the
   isotonic expected per diagonal (``sklearn.isotonic.IsotonicRegression(
   increasing='auto')`` on the balanced diagonal means — the reference's own
   call, :2022-2031) and the candidate pixels (nonzero raw contacts at
   ww <= d <= maxapart / res; the allelic gap / blanking filter, :1727-1759).
   O(N * num) glue.
2. GPU (``hh_hiccups_*``, csrc/loops.hip): the window-widening loop
   (:1776-1830) — donut and lower-left sums of the balanced and expected
   bands from per-row prefix sums, one launch per width; the host applies
   the reference's stop rule (< 10 % of the pending pixels became valid).
3. host: expected = EM * ratio * bias_i * bias_j, lambda chunks, Poisson
   p-values and Benjamini-Hochberg per chunk, q <= sig, the +-5-bin gap
   filter, donut AND lower-left (:1832-1948).  Vectorised; the p-values are
   computed once per distinct (observed count, chunk) and BH once per
   distinct p-value of a chunk — the same functions on the same inputs as
   the reference, so the results are identical.

Deviations (the reference raises): no candidate pixels, or every pixel valid
before the widening stops (its ratio divides by zero), return no calls.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import call, ptr


def peaks_parameter(res):
    """Peaks_Parameter (:1596-1615): dict(pw, ww, maxww, maxapart, sig)."""
    if res >= 20000:
        pw, ww = 1, 3
    elif res >= 10000:
        pw, ww = 2, 5
    else:
        pw, ww = 4, 7
    return dict(pw=pw, ww=ww, maxww=20, maxapart=2000000, sig=0.05)


def biases_from_weights(weights):
    """CallPeaks (:2007-2010): 1 / weight; weight == 0 -> 0; NaN stays NaN."""
    tmp = np.asarray(weights, dtype=np.float64)
    mask = np.logical_not(tmp == 0) | np.isnan(tmp)
    biases = np.zeros_like(tmp)
    biases[mask] = 1 / tmp[mask]
    return biases


def band_width(res, params=None):
    """``num`` of CallPeaks (:2020): diagonals 0 .. maxapart // res + maxww."""
    p = params or peaks_parameter(res)
    return p["maxapart"] // res + p["maxww"] + 1


def raw_band_from_pixels(bin1, bin2, count, lo, N, num):
    """raw[r, d] = H[r, r + d] (d < num) of chromosome bins [lo, lo + N)
    straight from cooler's upper-triangle pixel table (global ids, unique
    pixels): the band CallPeaks reads from ``matrix(balance=False).fetch``
    (:2006), without the N x N matrix."""
    b1 = np.asarray(bin1, dtype=np.int64) - lo
    b2 = np.asarray(bin2, dtype=np.int64) - lo
    c = np.asarray(count)
    d = b2 - b1
    k = (b1 >= 0) & (b1 < N) & (b2 < N) & (d >= 0) & (d < num)
    raw = np.zeros((N, num), dtype=c.dtype if c.dtype.kind in "iu" else np.float64)
    raw[b1[k], d[k]] = c[k]
    return raw


def bands(H_raw, weights, res, allelic=False, params=None, raw=None):
    """Raw / balanced bands, expected per diagonal and biases (:2003-2032),
    from the dense raw matrix or (``raw``, ``H_raw=None``) from its band."""
    p = params or peaks_parameter(res)
    num = band_width(res, p)
    if raw is None:
        H = np.asarray(H_raw)
        N = H.shape[0]
        r = np.arange(N)[:, None]
        d = np.arange(num)[None, :]
        raw = np.where((r + d) < N, H[r, np.minimum(r + d, N - 1)], 0)
    return _bands_from_raw(np.asarray(raw), weights, res, allelic, p)


def _bands_from_raw(raw, weights, res, allelic, p):
    from sklearn import isotonic
    ww = p["ww"]
    N, num = raw.shape
    r = np.arange(N)[:, None]
    d = np.arange(num)[None, :]
    inside = (r + d) < N
    cc = np.minimum(r + d, N - 1)
    if not allelic:
        w = np.asarray(weights, dtype=np.float64)
        # cH = nan_to_num(H * w_i * w_j), evaluated on the band in the same order
        bal = np.nan_to_num(raw.astype(float) * w[:, None] * np.where(inside, w[cc], 0.0))
        biases = biases_from_weights(w)
    else:
        bal = raw.astype(float)
        biases = np.ones(N)
    Hb = raw.astype(np.float64)
    Hb[:, 0] = 0.0                      # H - diag(H) (:2018)
    x = np.arange(ww, num)
    y = [bal[:N - i, i].mean() if i < N else np.nan for i in x]   # np.diagonal(cH, i).mean()
    IR = isotonic.IsotonicRegression(increasing="auto")
    IR.fit(x, y)
    pe = IR.predict(x)
    pe[pe < 0] = 0
    Eall = np.zeros(num)
    Eall[ww:] = pe
    Cb = np.where(d >= ww, bal, 0.0)
    return dict(N=N, num=num, res=res, allelic=allelic, Hb=np.ascontiguousarray(Hb),
                Cb=np.ascontiguousarray(Cb), Eall=Eall, biases=biases, **p)


def candidates(B, gap=None):
    """M.nonzero() with ww <= y - x <= maxapart // res (:1727-1730); for
    allelic data also the gap and blanking filter (:1731-1759), whose
    neighbour lookups follow the reference's dense-band indexing (row -1
    wraps to the last row; a column past the end counts as 1; `left` and
    `right` are the same cell)."""
    Hb, N, num = B["Hb"], B["N"], B["num"]
    rr, dd = np.nonzero(Hb)
    m = (dd >= B["ww"]) & (dd <= B["maxapart"] // B["res"])
    xi, yi = rr[m].astype(np.int64), (rr[m] + dd[m]).astype(np.int64)
    if B["allelic"]:
        def band(R, Cc):
            D = Cc - R
            ok = (D >= 0) & (D < num)
            v = np.zeros(R.shape)
            v[ok] = Hb[R[ok], D[ok]]
            return v
        gs = np.asarray(gap if gap is not None else [], dtype=np.int64)
        keep = ~(np.isin(xi, gs) & np.isin(yi, gs))
        left = band((xi - 1) % N, yi)
        top = np.where(yi + 1 >= N, 1.0, band(xi, np.minimum(yi + 1, N - 1)))
        bottom = band(xi, yi - 1)
        keep &= (left * left * top * bottom) != 0
        xi, yi = xi[keep], yi[keep]
    return xi, yi


class Neighbourhood:
    """Device state of one chromosome (``hh_hiccups``)."""

    def __init__(self, B, stream=None):
        _lib.require_gpu()
        self.B = B
        self.stream = stream
        h = C.c_void_p()
        call("hh_hiccups_create", ptr(B["Hb"]), ptr(B["Cb"]), ptr(np.ascontiguousarray(B["Eall"])), int(B["N"]),
             int(B["num"]), int(B["pw"]), 0, stream, C.byref(h))
        self._h = h

    def set_pixels(self, xi, yi):
        self.n = int(xi.size)
        r32 = np.ascontiguousarray(xi, dtype=np.int32)
        c32 = np.ascontiguousarray(yi, dtype=np.int32)
        call("hh_hiccups_set_pixels", self._h, ptr(r32), ptr(c32), self.n, self.stream)

    def widen(self):
        """The widening loop over the current pixels (all pending); returns
        [(w, newly valid, ratio)] with the reference's stop rule."""
        B = self.B
        pending = self.n
        widths = []
        for w in range(B["ww"], B["maxww"] + 1):
            if pending == 0:
                break  # the reference divides by zero here
            nv = C.c_int64(0)
            call("hh_hiccups_width", self._h, int(w), C.byref(nv), self.stream)
            ratio = nv.value / float(pending)
            pending -= nv.value
            widths.append((w, int(nv.value), ratio))
            if ratio < 0.1:
                break
        return widths

    def reset(self):
        call("hh_hiccups_reset", self._h, self.stream)

    def run(self, xi, yi):
        """The widening loop; returns (S, E, valid, widths) like the oracle."""
        self.set_pixels(xi, yi)
        widths = self.widen()
        n = self.n
        sK, sY, eK, eY = (np.empty(n) for _ in range(4))
        wid = np.empty(n, np.uint8)
        call("hh_hiccups_results", self._h, ptr(sK), ptr(sY), ptr(eK), ptr(eY), ptr(wid), self.stream)
        return {"K": sK, "Y": sY}, {"K": eK, "Y": eY}, wid != 0, widths

    def close(self):
        if getattr(self, "_h", None):
            call("hh_hiccups_free", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def lambda_chunks(E):
    """lambdachunk (:1617-1629) as (lv, rv) edges."""
    numbin = int(np.ceil(np.log(E.max()) / np.log(2) * 3 + 1))
    edges = []
    for i in range(1, numbin + 1):
        if i == 1:
            edges.append((0, 1))
        else:
            edges.append((np.power(2, ((i - 2) / 3.)), np.power(2, ((i - 1) / 3.))))
    return edges


def _bh_by_value(p):
    """statsmodels fdr_bh corrected p-values computed per distinct p-value
    (ties share a rank block; the reversed running minimum of p / (rank / n)
    over a block is its last rank's value)."""
    n = p.size
    u, inv, cnt = np.unique(p, return_inverse=True, return_counts=True)
    last = np.cumsum(cnt)                              # 1-based rank of each block's end
    ecdf = np.arange(1, n + 1) / float(n)              # statsmodels' ecdf factors
    raw = u / ecdf[last - 1]
    corr = np.minimum.accumulate(raw[::-1])[::-1]
    corr[corr > 1] = 1
    return corr[inv]


def significance(B, xi, yi, S, E, valid):
    """:1832-1948 -> (Donuts, LL) {(x*res, y*res): (O, fold, p, q)}."""
    from scipy.stats import poisson
    N, res, sig = B["N"], B["res"], B["sig"]
    mask = (E["K"] != 0) & (E["Y"] != 0) & valid
    xi, yi = xi[mask], yi[mask]
    gapind = (B["Hb"].sum(axis=1) == 0).astype(np.int64)
    gcum = np.concatenate([[0], np.cumsum(gapind)])
    res_fl = {}
    for fl in "KY":
        ratio = S[fl][mask] / E[fl][mask]
        cem = B["Eall"][yi - xi] * ratio
        nz = cem != 0
        x, y, cem = xi[nz], yi[nz], cem[nz]
        Ev = cem * B["biases"][x] * B["biases"][y]
        m = Ev > 0
        Ev, x, y = Ev[m], x[m], y[m]
        Ov = B["Hb"][x, y - x]
        fold = Ov / Ev
        pv = np.ones(x.size)
        qv = np.ones(x.size)
        edges = lambda_chunks(Ev) if Ev.size else []
        # no chunk at all when every expected value is below 2**(-2/3)
        # (numbin <= 0): the reference's lambdachunk Pool is empty, so p and q
        # stay 1 and nothing is called (StructureFind.py:1617-1629, :1866-1880)
        if edges:
            rvs = np.array([e[1] for e in edges], dtype=np.float64)
            lvs = np.array([e[0] for e in edges], dtype=np.float64)
            ci = np.searchsorted(rvs, Ev, side="right")        # first rv > E
            inchunk = ci < rvs.size
            ci_c = np.minimum(ci, rvs.size - 1)
            inchunk &= (Ev > lvs[ci_c]) & (Ev < rvs[ci_c])
            for c in np.unique(ci_c[inchunk]):
                idx = np.nonzero(inchunk & (ci_c == c))[0]
                ko, kinv = np.unique(Ov[idx], return_inverse=True)
                cp = (1 - poisson(edges[c][1]).cdf(ko))[kinv]
                pv[idx] = cp
                qv[idx] = _bh_by_value(cp)
        rej = qv <= sig
        x, y, Ov, fold, pv, qv = x[rej], y[rej], Ov[rej], fold[rej], pv[rej], qv[rej]
        if gapind.any():
            def lo_up(v):
                lo = np.where(v > 5, v - 5, 0)
                up = np.where(v + 5 < N, v + 5, N - 1)
                return lo, up
            l1, u1 = lo_up(x)
            l2, u2 = lo_up(y)
            hit = ((gcum[np.maximum(u1, l1)] - gcum[l1]) > 0) | ((gcum[np.maximum(u2, l2)] - gcum[l2]) > 0)
            keep = ~hit
            x, y, Ov, fold, pv, qv = x[keep], y[keep], Ov[keep], fold[keep], pv[keep], qv[keep]
        res_fl[fl] = (x * N + y, Ov, fold, pv, qv)
    kk, kc = res_fl["K"], res_fl["Y"]
    common, ia, ib = np.intersect1d(kk[0], kc[0], assume_unique=True, return_indices=True)
    Donuts, LL = {}, {}
    for j, lin in enumerate(common):
        pos = (int(lin // N) * res, int(lin % N) * res)
        a, b = ia[j], ib[j]
        Donuts[pos] = (kk[1][a], kk[2][a], kk[3][a], kk[4][a])
        LL[pos] = (kc[1][b], kc[2][b], kc[3][b], kc[4][b])
    return Donuts, LL


def pcaller(H_raw, weights, res, allelic=False, gap=None, stream=None, return_widths=False):
    """One chromosome of StructureFind.CallPeaks: (Donuts, LL) as the reference."""
    return _pcaller_bands(bands(H_raw, weights, res, allelic), gap, stream, return_widths)


def _pcaller_bands(B, gap=None, stream=None, return_widths=False):
    xi, yi = candidates(B, gap)
    nb = Neighbourhood(B, stream)
    try:
        S, E, valid, widths = nb.run(xi, yi)
    finally:
        nb.close()
    out = significance(B, xi, yi, S, E, valid)
    return out + (widths,) if return_widths else out


LINE_FORMAT = "%s\t%d\t%d\t%.4g\t%.4g\t%.4g\t%.4g\t%.4g\t%.4g\t%.4g\n"
HEAD = "\t".join(["chromLabel", "loc_1", "loc_2", "IF", "D-Enrichment", "D-pvalue", "D-qvalue",
                  "LL-Enrichment", "LL-pvalue", "LL-qvalue"]) + "\n"


def call_peaks_cooler(cooler_uri, outfil, res, allelic=False, gaps=None):
    """CallPeaks (:1954-2043) reading the cooler itself, as the reference
    does (:2003-2015): per chromosome the raw band from the pixel table
    (``matrix(balance=False)``), the balanced band from the same pixels and
    ``bins/weight`` (``matrix(balance=True)`` + nan_to_num, biases
    ``1 / weight``), allelic data raw with its gap list; no N x N matrix.
    ``allelic``: False, 'Maternal' or 'Paternal' (chromosomes by prefix)."""
    from .coolio import Cooler
    out = {}
    with Cooler(cooler_uri) as c:
        if allelic is False:
            chroms = list(c.chromnames)
        elif allelic in ("Maternal", "Paternal"):
            chroms = [x for x in c.chromnames if x.startswith(allelic[0])]
            if gaps is None:
                raise ValueError("Gap file needed for haplotype-resolved loop calling ...")
        else:
            raise ValueError(f"Unkonwn key word {allelic}, Only Maternal, Paternal, False allowed")
        w_all = c.weights() if allelic is False else None
        num = band_width(res)
        with open(outfil, "w") as f:
            f.write(HEAD)
            for chro in chroms:
                lo, hi = c.extent(chro)
                b1, b2, v = c.pixel_rows(lo, hi)
                raw = raw_band_from_pixels(b1, b2, v, lo, hi - lo, num)
                w = None if w_all is None else w_all[lo:hi]
                B = bands(None, w, res, allelic is not False, raw=raw)
                D, L = _pcaller_bands(B, None if allelic is False else gaps[chro])
                out[chro] = (D, L)
                label = chro if allelic is False else chro[1:]
                for pos in sorted(D):
                    f.write(LINE_FORMAT % ((label,) + pos + tuple(D[pos]) + tuple(L[pos][1:])))
    return out


def call_peaks(matrices, res, outfil, allelic=False, gaps=None):
    """CallPeaks (:1953-2043) over {chrom: (raw dense H, weights)}; writes the
    reference's tab-separated file (positions sorted; the reference's Python-2
    dict order is arbitrary).  Returns {chrom: (Donuts, LL)}."""
    out = {}
    with open(outfil, "w") as f:
        f.write(HEAD)
        for chro, (H, w) in matrices.items():
            D, L = pcaller(H, w, res, allelic, None if gaps is None else gaps[chro])
            out[chro] = (D, L)
            label = chro if not allelic else chro[1:]
            for pos in sorted(D):
                f.write(LINE_FORMAT % ((label,) + pos + tuple(D[pos]) + tuple(L[pos][1:])))
    return out


__all__ = ["peaks_parameter", "bands", "band_width", "raw_band_from_pixels", "call_peaks_cooler", "candidates", "Neighbourhood", "significance", "pcaller", "call_peaks",
           "lambda_chunks", "biases_from_weights"]
