"""ORACLE (test infrastructure only) — cooler ICE balancing, restated in NumPy.

HiCHap does not implement ICE itself: it shells out to the third-party
``cooler`` CLI, ``cooler balance --ignore-diags 1 [--cis-only] --force
<file>::<res>`` (matrixBuilding.py:708, :713, :1537, :1542, :1761, :1766).
``cooler`` is not vendored in /root/reference, its version is not pinned
(setup.py has no install_requires; README.md:27 names it only) and it is not
installed in this image.

PARITY UNPINNED: no golden vector from the reference covers this function.
This module restates cooler's published ``balance_cooler`` algorithm
(cooler/balance.py: ``_binarize``, ``_zero_diags``, ``_zero_trans``,
``_timesouterproduct``, ``_marginalize``, MAD filter, ``_balance_genomewide``
/ ``_balance_cisonly``) as summarised in SURVEY.md Appendix B, and is pinned by
analytic known-answer tests in tests/test_oracle_ice.py (D·K·D recovery,
balanced marginals == 1, masking rules).

Inputs are the cooler pixel table (upper triangle, ``bin1 <= bin2``) plus the
chromosome bin offsets (``indexes/chrom_offset``).
"""
from __future__ import annotations

import numpy as np

DEFAULTS = dict(ignore_diags=1, cis_only=False, mad_max=5, min_nnz=10, min_count=0,
                tol=1e-5, max_iters=200, rescale_marginals=True)


def _mad(x):
    """Median absolute deviation (cooler.balance.mad)."""
    return np.median(np.abs(x - np.median(x)))


def _active_pixels(bin1, bin2, count, chrom_of, ignore_diags, cis_only):
    """Apply the static filters (zero_trans, zero_diags); return kept pixels."""
    keep = np.ones(bin1.shape, dtype=bool)
    if cis_only:
        keep &= chrom_of[bin1] == chrom_of[bin2]
    if ignore_diags:
        keep &= np.abs(bin2 - bin1) >= ignore_diags
    return bin1[keep], bin2[keep], count[keep].astype(np.float64)


def marginalize(bin1, bin2, w, n):
    """``bincount(bin1, w) + bincount(bin2, w)`` (cooler ``_marginalize``)."""
    return (np.bincount(bin1, weights=w, minlength=n)
            + np.bincount(bin2, weights=w, minlength=n))


def ice_filters(bin1, bin2, count, n_bins, chrom_offsets, ignore_diags=1, cis_only=False,
                mad_max=5, min_nnz=10, min_count=0):
    """Initial bias after cooler's bad-bin filters. Returns (bias, pixels)."""
    chrom_offsets = np.asarray(chrom_offsets, dtype=np.int64)
    chrom_of = np.repeat(np.arange(len(chrom_offsets) - 1), np.diff(chrom_offsets))
    b1, b2, c = _active_pixels(np.asarray(bin1, np.int64), np.asarray(bin2, np.int64),
                               np.asarray(count), chrom_of, ignore_diags, cis_only)
    bias = np.ones(n_bins, dtype=np.float64)
    if min_nnz > 0:
        nnz_marg = marginalize(b1, b2, (c != 0).astype(np.float64), n_bins)
        bias[nnz_marg < min_nnz] = 0
    marg = marginalize(b1, b2, c, n_bins)
    if min_count:
        bias[marg < min_count] = 0
    if mad_max > 0:
        marg = marg.copy()
        with np.errstate(invalid="ignore", divide="ignore"):
            for lo, hi in zip(chrom_offsets[:-1], chrom_offsets[1:]):
                cm = marg[lo:hi]
                pos = cm[cm > 0]
                med = np.median(pos) if pos.size else np.nan
                marg[lo:hi] = cm / med
            logm = np.log(marg[marg > 0])
            cutoff = np.exp(np.median(logm) - mad_max * _mad(logm))
            bias[marg < cutoff] = 0
    return bias, (b1, b2, c)


def _iterate(bias, b1, b2, c, n, lo, hi, tol, max_iters):
    """ICE sweeps restricted to bins [lo, hi); mutates ``bias``.

    Returns (scale, var, n_iters, converged)."""
    var = np.nan
    nzmarg = None
    it = 0
    converged = False
    for it in range(1, max_iters + 1):
        marg = marginalize(b1, b2, c * bias[b1] * bias[b2], n)[lo:hi]
        nzmarg = marg[marg != 0]
        if nzmarg.size == 0:
            bias[lo:hi] = np.nan
            return np.nan, 0.0, it, True
        m = marg / nzmarg.mean()
        m[m == 0] = 1
        bias[lo:hi] /= m
        var = nzmarg.var()
        if var < tol:
            converged = True
            break
    scale = nzmarg.mean()
    return scale, var, it, converged


def balance(bin1, bin2, count, n_bins, chrom_offsets, ignore_diags=1, cis_only=False,
            mad_max=5, min_nnz=10, min_count=0, tol=1e-5, max_iters=200,
            rescale_marginals=True):
    """cooler ``balance_cooler`` restated. Returns ``(weights, stats)``.

    ``stats`` mirrors the attrs cooler writes on ``bins/weight``; in cis-only
    mode ``scale`` is the per-chromosome scale array and ``var`` the last
    chromosome's variance (as cooler returns them), ``iters`` per chromosome.
    """
    bias, (b1, b2, c) = ice_filters(bin1, bin2, count, n_bins, chrom_offsets,
                                    ignore_diags, cis_only, mad_max, min_nnz, min_count)
    chrom_offsets = np.asarray(chrom_offsets, dtype=np.int64)
    if cis_only:
        scales = np.ones(len(chrom_offsets) - 1)
        iters = np.zeros(len(chrom_offsets) - 1, dtype=np.int64)
        conv = np.zeros(len(chrom_offsets) - 1, dtype=bool)
        var = np.nan
        for k, (lo, hi) in enumerate(zip(chrom_offsets[:-1], chrom_offsets[1:])):
            sel = (b1 >= lo) & (b1 < hi)
            scale, var, it, cv = _iterate(bias, b1[sel], b2[sel], c[sel], n_bins,
                                          lo, hi, tol, max_iters)
            seg = bias[lo:hi]
            seg[seg == 0] = np.nan
            scales[k] = scale
            iters[k] = it
            conv[k] = cv
            if rescale_marginals:
                bias[lo:hi] = seg / np.sqrt(scale)
        stats = dict(tol=tol, min_nnz=min_nnz, min_count=min_count, mad_max=mad_max,
                     cis_only=True, ignore_diags=ignore_diags, scale=scales,
                     converged=bool(var < tol) if var == var else False, var=var,
                     divisive_weights=False, iters=iters, chrom_converged=conv)
        return bias, stats
    scale, var, it, cv = _iterate(bias, b1, b2, c, n_bins, 0, n_bins, tol, max_iters)
    bias[bias == 0] = np.nan
    if rescale_marginals:
        bias /= np.sqrt(scale)
    stats = dict(tol=tol, min_nnz=min_nnz, min_count=min_count, mad_max=mad_max,
                 cis_only=False, ignore_diags=ignore_diags, scale=scale,
                 converged=bool(var < tol), var=var, divisive_weights=False, iters=it)
    return bias, stats


def sweep_rate(bin1, bin2, count, n_bins, iters):
    """CPU-baseline timing helper: run ``iters`` un-filtered ICE sweeps (the
    timed loop of cooler ``_balance_genomewide``) and return the bias."""
    b1 = np.asarray(bin1, np.int64)
    b2 = np.asarray(bin2, np.int64)
    c = np.asarray(count, np.float64)
    bias = np.ones(n_bins)
    for _ in range(iters):
        marg = marginalize(b1, b2, c * bias[b1] * bias[b2], n_bins)
        nz = marg[marg != 0]
        m = marg / nz.mean()
        m[m == 0] = 1
        bias /= m
        _ = nz.var()
    return bias


# ------------------------------------------------ process-pool CPU baseline
# cooler's balance splits each sweep over a process pool (``cooler balance
# --nproc``, default 8): every worker marginalises its chunks of the pixel
# table with the current bias, the parent sums the partial vectors.  The
# same here, for bench.py's multi-core CPU baseline (test infrastructure):
# forked workers, the pixel table inherited, the bias and the partial
# marginals in shared memory (no per-task pickling of 5 MB vectors).
_POOL = None


def _pool_chunk(k):
    b1, b2, c, n, cuts, bias_sh, out_sh = _POOL
    lo, hi = int(cuts[k]), int(cuts[k + 1])
    bias = np.frombuffer(bias_sh, dtype=np.float64)
    out = np.frombuffer(out_sh, dtype=np.float64).reshape(-1, n)
    s1, s2 = b1[lo:hi], b2[lo:hi]
    out[k] = marginalize(s1, s2, c[lo:hi] * bias[s1] * bias[s2], n)
    return k


def sweep_rate_pool(bin1, bin2, count, n_bins, iters, nproc):
    """``sweep_rate`` with each sweep's marginal split over ``nproc`` forked
    processes (cooler's balance pool), one pixel chunk each, the partials
    summed in chunk order.  Returns the bias."""
    import multiprocessing as mp
    global _POOL
    n = int(n_bins)
    nch = max(1, int(nproc))
    b1 = np.asarray(bin1, np.int64)
    b2 = np.asarray(bin2, np.int64)
    c = np.asarray(count, np.float64)
    cuts = np.linspace(0, b1.size, nch + 1).astype(np.int64)
    bias_sh = mp.RawArray("d", n)
    out_sh = mp.RawArray("d", nch * n)
    bias = np.frombuffer(bias_sh, dtype=np.float64)
    out = np.frombuffer(out_sh, dtype=np.float64).reshape(nch, n)
    bias[:] = 1.0
    _POOL = (b1, b2, c, n, cuts, bias_sh, out_sh)
    try:
        with mp.get_context("fork").Pool(nch) as pool:
            for _ in range(iters):
                pool.map(_pool_chunk, range(nch), chunksize=1)
                marg = out[0].copy()
                for q in range(1, nch):
                    marg += out[q]
                nz = marg[marg != 0]
                m = marg / nz.mean()
                m[m == 0] = 1
                bias /= m
                _ = nz.var()
        return bias.copy()
    finally:
        _POOL = None
