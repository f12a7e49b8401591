"""Synthetic Hi-C contact matrices (host side, NumPy).

Shapes follow SURVEY.md §8(d): per chromosome with n bins the expected
contact frequency is

    lambda(i, j) = A * (|j - i| + 1) ** -1.08 * (1 + 0.3 * s_i * s_j) * v_i * v_j

with ``s`` = +/-1 compartment blocks, ``v`` ~ LogNormal(0, 0.3) visibility and
~2 % of bins zeroed (gaps); counts ~ Poisson(lambda).  Trans (inter-chromosome)
contacts are uniform with a fixed density.

These generators are used for the CPU-sized configs (C1, parity fixtures) and
for tests.  The 5e9-pixel whole-genome config (C4) is generated on the device
(``hh_synth_*`` in the C-ABI) because it is 60 GB as a host COO.
"""
from __future__ import annotations

import numpy as np

# hg19 chromosome lengths, chr1-22 + X (public assembly facts).
HG19 = {
    "1": 249250621, "2": 243199373, "3": 198022430, "4": 191154276,
    "5": 180915260, "6": 171115067, "7": 159138663, "8": 146364022,
    "9": 141213431, "10": 135534747, "11": 135006516, "12": 133851895,
    "13": 115169878, "14": 107349540, "15": 102531392, "16": 90354753,
    "17": 81195210, "18": 78077248, "19": 59128983, "20": 63025520,
    "21": 48129895, "22": 51304566, "X": 155270560,
}


def chrom_bins(lengths, res):
    """Bins per chromosome as HiCHap counts them: ``l // res + 1``
    (matrixBuilding.py:564, :416-422)."""
    return [int(l) // int(res) + 1 for l in lengths]


def bin_profile(n, rng, gap_frac=0.02, comp_len=(5, 15)):
    """Per-bin compartment sign ``s``, visibility ``v`` and gap mask."""
    s = np.empty(n, dtype=np.float64)
    i = 0
    sign = 1.0 if rng.random() < 0.5 else -1.0
    while i < n:
        L = int(rng.integers(comp_len[0], comp_len[1] + 1))
        s[i:i + L] = sign
        sign = -sign
        i += L
    v = np.exp(rng.normal(0.0, 0.3, size=n))
    gap = rng.random(n) < gap_frac
    v[gap] = 0.0
    return s, v, gap


def dense_chrom(n, rng, A=50.0, max_dist=None, gap_frac=0.02, comp_len=(5, 15)):
    """Symmetric int64 dense contact matrix for one chromosome."""
    s, v, gap = bin_profile(n, rng, gap_frac, comp_len)
    i = np.arange(n)
    d = np.abs(i[:, None] - i[None, :])
    lam = A * (d + 1.0) ** -1.08 * (1.0 + 0.3 * s[:, None] * s[None, :]) * v[:, None] * v[None, :]
    if max_dist is not None:
        lam[d > max_dist] = 0.0
    up = rng.poisson(np.triu(lam))
    M = np.triu(up) + np.triu(up, 1).T
    return M.astype(np.int64)


def haplotype_pair(TM, rng, frac=0.4, asym=0.15, drop_rows=0):
    """Maternal / paternal matrices derived from a traditional matrix.

    Allele-resolved reads are a thinned subset of the traditional reads; R1/R2
    imputation makes MM and PM asymmetric (matrixBuilding.py:1290-1301), which
    is modelled by a one-sided extra thinning of the upper triangle.
    ``drop_rows`` rows/cols are made nearly empty to create SNP-poor gaps.
    """
    n = TM.shape[0]
    base = rng.binomial(TM, frac)
    MM = rng.binomial(base, 0.5)
    PM = base - MM
    for X in (MM, PM):
        extra = rng.binomial(np.triu(X, 1), asym)
        X -= extra
    if drop_rows:
        for X in (MM, PM):
            rows = rng.choice(n, size=drop_rows, replace=False)
            X[rows, :] = rng.binomial(X[rows, :], 0.02)
            X[:, rows] = rng.binomial(X[:, rows], 0.02)
    return MM.astype(np.int64), PM.astype(np.int64)


def coo_genome(nbins_per_chrom, rng, A=30.0, max_dist=None, trans_density=0.0,
               gap_frac=0.02, comp_len=(5, 15), count_dtype=np.int32):
    """Upper-triangle COO (bin1 <= bin2, sorted by bin1 then bin2) for a genome
    made of chromosomes with the given bin counts, cooler pixel-table layout.

    Returns ``(bin1, bin2, count, chrom_offsets)`` with int64 ids.
    """
    offsets = np.concatenate([[0], np.cumsum(nbins_per_chrom)]).astype(np.int64)
    n = int(offsets[-1])
    s = np.empty(n)
    v = np.empty(n)
    for c in range(len(nbins_per_chrom)):
        lo, hi = offsets[c], offsets[c + 1]
        s[lo:hi], v[lo:hi], _ = bin_profile(hi - lo, rng, gap_frac, comp_len)
    b1s, b2s, cs = [], [], []
    for c in range(len(nbins_per_chrom)):
        lo, hi = int(offsets[c]), int(offsets[c + 1])
        L = hi - lo
        dmax = L - 1 if max_dist is None else min(L - 1, max_dist)
        for d in range(0, dmax + 1):
            i = np.arange(lo, hi - d)
            j = i + d
            lam = A * (d + 1.0) ** -1.08 * (1.0 + 0.3 * s[i] * s[j]) * v[i] * v[j]
            k = rng.poisson(lam)
            nz = k > 0
            b1s.append(i[nz]); b2s.append(j[nz]); cs.append(k[nz])
    if trans_density > 0 and len(nbins_per_chrom) > 1:
        chrom_of = np.repeat(np.arange(len(nbins_per_chrom)), nbins_per_chrom)
        # number of trans pixels in the upper triangle
        sizes = np.asarray(nbins_per_chrom, dtype=np.float64)
        n_trans_pos = (n * n - (sizes * sizes).sum()) / 2.0
        m = rng.poisson(trans_density * n_trans_pos)
        a = rng.integers(0, n, size=int(m * 1.2) + 16)
        b = rng.integers(0, n, size=a.size)
        lo_, hi_ = np.minimum(a, b), np.maximum(a, b)
        keep = chrom_of[lo_] != chrom_of[hi_]
        lo_, hi_ = lo_[keep][:m], hi_[keep][:m]
        key = np.unique(lo_ * n + hi_)
        lo_, hi_ = key // n, key % n
        vis = v[lo_] * v[hi_]
        keep = vis > 0
        lo_, hi_ = lo_[keep], hi_[keep]
        k = 1 + rng.poisson(0.3, size=lo_.size)
        b1s.append(lo_); b2s.append(hi_); cs.append(k)
    bin1 = np.concatenate(b1s).astype(np.int64)
    bin2 = np.concatenate(b2s).astype(np.int64)
    count = np.concatenate(cs).astype(count_dtype)
    order = np.lexsort((bin2, bin1))
    return bin1[order], bin2[order], count[order], offsets


def coo_to_dense(bin1, bin2, count, n):
    """Symmetric dense matrix from an upper-triangle COO (like cooler's
    ``matrix(balance=False)[:]``)."""
    M = np.zeros((n, n), dtype=np.float64)
    M[bin1, bin2] = count
    M[bin2, bin1] = count
    return M


# ----------------------------------------------------- device-generator model
HG19_ORDER = [str(i) for i in range(1, 23)] + ["X"]


def genome_bins(res, diploid=False, chroms=None):
    """Per-chromosome bin counts (HiCHap's ``l // res + 1``) for hg19 chr1-22,X;
    diploid = maternal copies then paternal copies (matrixBuilding.py:429-454)."""
    chroms = chroms or HG19_ORDER
    nb = chrom_bins([HG19[c] for c in chroms], res)
    return nb + nb if diploid else nb


def _modulation_samples(k=4096, vis_sigma=0.3, comp=0.3, seed=0):
    rng = np.random.default_rng(seed)
    v = np.exp(vis_sigma * rng.normal(size=(2, k)))
    s = np.where(rng.random(k) < 0.5, 1.0 + comp, 1.0 - comp)
    return v[0] * v[1] * s, float(np.mean(v[0] * v[1]))


def expected_nnz(chrom_nbins, A, trans_density=0.0, decay=1.08, vis_sigma=0.3, comp=0.3,
                 gap_frac=0.02, ignore_diags=1):
    """Expected upper-triangle pixel count of the device generator's model
    (hh_synth_*): sum over cis distances of P(Poisson(lambda) > 0), plus the
    uniform trans density.  Used to pick ``A`` for a target nnz."""
    nb = np.asarray(chrom_nbins, dtype=np.int64)
    m, ev = _modulation_samples(vis_sigma=vis_sigma, comp=comp)
    L = int(nb.max())
    d = np.arange(max(ignore_diags, 1), L)
    # pairs at distance d summed over chromosomes
    pairs = np.zeros(d.size)
    for Lc in nb:
        pairs[: max(Lc - d[0], 0)] += Lc - d[: max(Lc - d[0], 0)]
    # P(count > 0) is smooth in d: evaluate on a log grid and interpolate
    grid = np.unique(np.round(np.geomspace(d[0], d[-1] if d.size else 1, 256)).astype(np.int64))
    lam = A * (grid[:, None] + 1.0) ** -decay * m[None, :]
    pg = np.mean(-np.expm1(-lam), axis=1)
    p = np.interp(d, grid, pg)
    keep = (1 - gap_frac) ** 2
    cis = float(np.sum(pairs * p)) * keep
    tot = float(nb.sum())
    trans_pairs = (tot * tot - float(np.sum(nb.astype(np.float64) ** 2))) / 2.0
    trans = trans_density * ev * keep * trans_pairs
    return cis, trans


def calibrate(chrom_nbins, target_nnz, trans_frac=0.0, **kw):
    """(A, trans_density) whose expected nnz is ``target_nnz`` with the given
    trans fraction."""
    nb = np.asarray(chrom_nbins, dtype=np.float64)
    _, ev = _modulation_samples()
    keep = (1 - kw.get("gap_frac", 0.02)) ** 2
    trans_pairs = (nb.sum() ** 2 - np.sum(nb ** 2)) / 2.0
    tdens = trans_frac * target_nnz / (ev * keep * trans_pairs) if trans_frac > 0 else 0.0
    want = target_nnz * (1.0 - trans_frac)
    lo, hi = 1e-2, 1e6
    for _ in range(48):
        mid = np.sqrt(lo * hi)
        c, _ = expected_nnz(chrom_nbins, mid, 0.0, **kw)
        lo, hi = (mid, hi) if c < want else (lo, mid)
    return float(np.sqrt(lo * hi)), float(tdens)
