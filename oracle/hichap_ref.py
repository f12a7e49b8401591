"""ORACLE (test infrastructure only) — HiCHap's two-step / genome-wide bias
correction restated in vectorised NumPy.

Pinned against golden vectors produced by the reference's own functions
(tests/golden/make_golden.py, fixtures tests/golden/twostep_*.npz and
genomewide_*.npz).  Every function cites the reference lines it restates.
"""
from __future__ import annotations

import numpy as np

VC_EXPONENT = 2 / 3  # Correct_VC(X, 2/3) with true division (matrixBuilding.py:8, :1014)


def coverage(M):
    """Fraction of nonzero entries per row (Coverage_M, matrixBuilding.py:904-912)."""
    M = np.asarray(M)
    return 1 - (M == 0).sum(axis=1) / float(M.shape[1])


def gap_defined(M):
    """Gap rows: coverage < min(25th percentile of nonzero coverage, 0.2)
    (Gap_defined, matrixBuilding.py:915-929). Returns sorted int64 indices."""
    cov = coverage(M)
    thr = min(np.percentile(cov[np.nonzero(cov)], 25), 0.2)
    return np.nonzero(cov < thr)[0].astype(np.int64)


def gap_defined_lowres(M):
    """Gap rows with fixed threshold 0.1 (Gap_definedLowRes, :742-753)."""
    return np.nonzero(coverage(M) < 0.1)[0].astype(np.int64)


def non_gap(N, gap):
    """Complement of ``gap`` in range(N) (Non_Gap_Defined, :932-942)."""
    mask = np.ones(N, dtype=bool)
    mask[np.asarray(gap, dtype=np.int64)] = False
    return np.nonzero(mask)[0].astype(np.int64)


def symmetrize(S, gap):
    """Gap-aware symmetrisation (Trans2symmetry, :945-979).

    No gap: Y_ij = S_ij + S_ji off-diagonal (a sum).  Otherwise a pair with at
    least one non-gap end is averaged, a gap-gap pair takes the max; the
    diagonal is kept."""
    S = np.asarray(S, dtype=np.float64)
    N = S.shape[0]
    gap = np.asarray(gap)
    if gap.size == 0:
        Y = S + S.T
    else:
        g = np.zeros(N, dtype=bool)
        g[gap] = True
        both_gap = g[:, None] & g[None, :]
        Y = np.where(both_gap, np.maximum(S, S.T), (S + S.T) / 2.0)
    np.fill_diagonal(Y, np.diag(S))
    return Y


def symmetrize_sum(S):
    """Trans2symmetryLowRes (:770-777): off-diagonal S_ij + S_ji, diagonal kept."""
    S = np.asarray(S, dtype=np.float64)
    Y = S + S.T
    np.fill_diagonal(Y, np.diag(S))
    return Y


def correct_vc(X, alpha=VC_EXPONENT):
    """Vanilla-coverage rescale (Correct_VC, :780-790)."""
    x = np.array(X, dtype=np.float64)
    r = np.sum(x, axis=1) ** alpha
    r[r == 0] = 1
    c = np.sum(x, axis=0) ** alpha
    c[c == 0] = 1
    return x / (c[None, :] * r[:, None])


def snp_alpha(T, M, P, nongap):
    """SNP-density factor (TwoStepCorrection :989-1005 / GenomeWide :878-886)."""
    alpha = (M.sum(axis=1) + P.sum(axis=1)) / (T.sum(axis=1) + 1)
    alpha = alpha.astype(np.float64)
    alpha /= np.max(alpha[nongap])
    alpha[alpha == 0] = 1
    thr = np.percentile(alpha[nongap], 20)
    alpha[alpha < thr] = thr
    return alpha


def two_step_correction(TM, MM, PM):
    """TwoStepCorrection (matrixBuilding.py:984-1023).
    Returns (Nor_MM, Nor_PM, Gap_M, Gap_P)."""
    N = TM.shape[0]
    gm, gp = gap_defined(MM), gap_defined(PM)
    ng = np.union1d(non_gap(N, gm), non_gap(N, gp))
    alpha = snp_alpha(TM, MM, PM, ng)
    out = []
    for X, g in ((MM, gm), (PM, gp)):
        Y = symmetrize(X / alpha[:, None], g)
        C = correct_vc(Y)
        out.append((X.mean() / C.mean()) * C)
    return out[0], out[1], gm, gp


def sort_chromosomes(names):
    """Numeric labels ascending, then string labels sorted (Sort_Chromosomes,
    :388-406); a leading 'chr' is stripped."""
    names = [n[3:] if n.startswith("chr") else n for n in names]
    num = sorted(int(n) for n in names if n.lstrip("-").isdigit())
    txt = sorted(n for n in names if not n.lstrip("-").isdigit())
    return [str(n) for n in num] + txt


def genome_wide_correction(bins_pos, hap_bins_pos, T_M, H_M):
    """GenomeWideMatrixCorrection (matrixBuilding.py:857-901).

    ``bins_pos[chrom] = (start, end)`` inclusive bin ranges in T_M;
    ``hap_bins_pos['M'+chrom]`` / ``['P'+chrom]`` the same in H_M."""
    alphas = {}
    for c, (s, e) in bins_pos.items():
        T = T_M[s:e + 1, s:e + 1]
        ms, me = hap_bins_pos["M" + c]
        ps, pe = hap_bins_pos["P" + c]
        Mb = H_M[ms:me + 1, ms:me + 1]
        Pb = H_M[ps:pe + 1, ps:pe + 1]
        g = gap_defined_lowres(T)
        alphas[c] = snp_alpha(T, Mb, Pb, non_gap(T.shape[0], g))
    alpha = np.concatenate([alphas[c] for c in sort_chromosomes(list(alphas))])
    alpha = np.concatenate([alpha, alpha])
    Y = symmetrize_sum(H_M / alpha[:, None])
    C = correct_vc(Y)
    return (H_M.mean() / C.mean()) * C


def genome_wide_correction_sparse(bins_pos, hap_bins_pos, T_pixels, H_cells):
    """GenomeWideMatrixCorrection (matrixBuilding.py:857-901) restated on
    pixel tables, for whole-genome diploid sizes the dense form cannot hold
    (10 kb: 607 282^2 x 8 B = 2.9 TB).  ``T_pixels`` = cooler's upper-triangle
    table of T_M, ``H_cells`` = the nonzero ordered cells of the asymmetric
    H_M.  Same arithmetic as :func:`genome_wide_correction`: block row sums of
    T (Gap_definedLowRes coverage, :742-753) and of the M_M / P_P blocks of H
    (:878-886, exact integers), Alpha in Sort_Chromosomes order and duplicated
    (:887-892), S = H / Alpha[:, None], the sum symmetrisation
    (Trans2symmetryLowRes, :770-777: Y_ij = S_ij + S_ji, diagonal kept),
    Correct_VC(Y, 2/3) (:780-790) and the mean rescale (:897-899).  Returns
    the upper triangle (bin1, bin2, value), sorted and unique (cooler order)."""
    t1, t2, tv = (np.asarray(x) for x in T_pixels)
    t1, t2, tv = t1.astype(np.int64), t2.astype(np.int64), tv.astype(np.int64)
    hr, hc, hv = (np.asarray(x) for x in H_cells)
    hr, hc, hv = hr.astype(np.int64), hc.astype(np.int64), hv.astype(np.int64)
    names = list(bins_pos)
    n = max(e for _, e in bins_pos.values()) + 1
    N2 = 2 * n
    chrom_of = np.full(n, -1, np.int64)
    for k, c in enumerate(names):
        s, e = bins_pos[c]
        chrom_of[s:e + 1] = k
    # T row sums / nonzeros within each chromosome block (both triangles, diagonal once)
    cis = chrom_of[t1] == chrom_of[t2]
    off = cis & (t1 != t2)
    tsum = np.bincount(t1[cis], tv[cis], minlength=n) + np.bincount(t2[off], tv[off], minlength=n)
    tsum = np.rint(tsum).astype(np.int64)
    nzc, nzo = cis & (tv != 0), off & (tv != 0)
    tnz = np.bincount(t1[nzc], minlength=n) + np.bincount(t2[nzo], minlength=n)
    # H row sums within the M_M / P_P block of the row's chromosome copy
    block_of = np.full(N2, -1, np.int64)
    for k, c in enumerate(names):
        for h, key in ((0, "M" + c), (1, "P" + c)):
            s, e = hap_bins_pos[key]
            block_of[s:e + 1] = 2 * k + h
    same = block_of[hr] == block_of[hc]
    hbs = np.rint(np.bincount(hr[same], hv[same], minlength=N2)).astype(np.int64)  # exact below 2^53
    alphas = {}
    for c in names:
        s, e = bins_pos[c]
        L = e - s + 1
        cov = 1 - (L - tnz[s:e + 1]) / float(L)
        gap = np.nonzero(cov < 0.1)[0]
        ms, me = hap_bins_pos["M" + c]
        ps, pe = hap_bins_pos["P" + c]
        alpha = (hbs[ms:me + 1] + hbs[ps:pe + 1]) / (tsum[s:e + 1] + 1)
        alpha = alpha.astype(np.float64)
        ng = non_gap(L, gap)
        alpha /= np.max(alpha[ng])
        alpha[alpha == 0] = 1
        thr = np.percentile(alpha[ng], 20)
        alpha[alpha < thr] = thr
        alphas[c] = alpha
    Alpha = np.concatenate([alphas[c] for c in sort_chromosomes(names)])
    Alpha = np.concatenate([Alpha, Alpha])
    S = hv / Alpha[hr]
    # Y upper table: S_rc at key (min, max); partners add, the diagonal stays single
    lo, hi = np.minimum(hr, hc), np.maximum(hr, hc)
    key = lo * N2 + hi
    o = np.argsort(key, kind="stable")
    ks, vs = key[o], S[o]
    first = np.concatenate([[True], ks[1:] != ks[:-1]]) if ks.size else np.zeros(0, bool)
    idx = np.flatnonzero(first)
    ukey = ks[idx]
    Y = np.add.reduceat(vs, idx) if ks.size else np.zeros(0)
    b1, b2 = ukey // N2, ukey % N2
    offd = b1 != b2
    rs = np.bincount(b1, Y, minlength=N2) + np.bincount(b2[offd], Y[offd], minlength=N2)
    sv = rs ** VC_EXPONENT
    sv[sv == 0] = 1
    C = Y / (sv[b2] * sv[b1])
    csum = np.sum(np.where(offd, 2.0, 1.0) * C)
    NN = float(N2) * float(N2)
    rf = (float(hv.sum()) / NN) / (csum / NN)
    return b1, b2, rf * C
