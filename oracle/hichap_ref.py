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
