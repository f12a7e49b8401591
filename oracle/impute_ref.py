"""CPU oracle for the haplotype imputation of HaplotypeMatrixBuilding (test
infrastructure only: imported by tests/ and bench.py's cpu_baseline leg).

Restates HiCHap/matrixBuilding.py:1251-1494 line by line, bugs included:

* only single-allele lines (last field != 'Both') of the M_M and P_P beds;
  intra-chromosome ones add one count to the imputed whole / local matrix at
  (bin1, bin2) for 'R1', else at (bin2, bin1) — asymmetric;
* inter-chromosome ones compare two neighbourhood sums of the UNIMPUTED
  whole matrix (GetNeighborhoodIndex :721-732: the disc d^2 < L around
  (L+1, L+1) of a (2L+1)^2 window, L = Imputation_region // res) and impute
  when a sum >= Imputation_min holds > Imputation_ratio of both;
* 'R2' lines take chrom1's offset for pos2 and chrom2's for pos1 (:1347-1349);
* the P pass's 'R1' branch sums the stale ``M_M_sub`` left by the last M-pass
  line that reached the window step (:1445), and adds to the M copy of
  chrom2 when that sum wins (:1451) — no such line: the reference raises
  NameError (so does this).

Pinned by tests/golden/impute_*.npz (tests/golden/make_golden_impute.py runs
the reference's own statements).
"""
from __future__ import annotations

import math

import numpy as np

from .pairs_ref import _passes, get_chro_bins_haplotypes


def neighborhood_index(L):
    """GetNeighborhoodIndex (:721-732)."""
    center = L + 1
    ii, jj = [], []
    for i in range(L * 2 + 1):
        for j in range(L * 2 + 1):
            if math.sqrt((i - center) ** 2 + (j - center) ** 2) < math.sqrt(L):
                ii.append(i)
                jj.append(j)
    return ii, jj


def impute(sources, genome, chroms, wholeRes, localRes, region, imin, iratio, UW, UL):
    """sources = {'M_M': lines, 'P_P': lines}; UW[res] dense 2n x 2n unimputed
    whole matrix, UL[res][hap+chrom] dense unimputed local matrices.
    Returns (IW, IL) dense copies with the imputed counts added."""
    IW = {res: np.array(UW[res], dtype=np.int64, copy=True) for res in wholeRes}
    IL = {res: {k: np.array(v, dtype=np.int64, copy=True) for k, v in UL[res].items()} for res in localRes}
    pos_of, sub, idx = {}, {}, {}
    for res in wholeRes:
        pos_of[res] = get_chro_bins_haplotypes(genome, res)[0]
        sub[res] = region // res
        idx[res] = neighborhood_index(sub[res])
    stale = None  # M_M_sub: a name of the reference's function scope
    for hap, kind in (("M", "M_M"), ("P", "P_P")):
        for line in sources.get(kind, []):
            line = line.strip().split()
            mark = line[-1]
            if mark == "Both":
                continue
            c1 = line[0].lstrip("chr")
            c2 = line[2].lstrip("chr")
            if not (_passes(c1, chroms) and _passes(c2, chroms)):
                continue
            if c1 == c2:
                for res in wholeRes:
                    p1, p2 = int(line[1]) // res, int(line[3]) // res
                    b1 = p1 + pos_of[res][hap + c1][0]
                    b2 = p2 + pos_of[res][hap + c2][0]
                    if mark == "R1":
                        _inc(IW[res], b1, b2)
                    else:
                        _inc(IW[res], b2, b1)
                for res in localRes:
                    p1, p2 = int(line[1]) // res, int(line[3]) // res
                    if mark == "R1":
                        _inc(IL[res][hap + c1], p1, p2)
                    else:
                        _inc(IL[res][hap + c2], p2, p1)
                continue
            for res in wholeRes:
                p1, p2 = int(line[1]) // res, int(line[3]) // res
                P = pos_of[res]
                s = sub[res]
                Mx = UW[res]
                n = Mx.shape[0]
                ii, jj = idx[res]
                if mark == "R1":
                    a = p1 + P[hap + c1][0]
                    mb, pb = p2 + P["M" + c2][0], p2 + P["P" + c2][0]
                    if a < s or mb < s or pb < s or a + s + 1 > n or mb + s + 1 > n or pb + s + 1 > n:
                        continue
                    if hap == "M":
                        stale = Mx[a - s:a + s + 1, mb - s:mb + s + 1]
                        own = stale[ii, jj].sum()
                        other = Mx[a - s:a + s + 1, pb - s:pb + s + 1][ii, jj].sum()
                        cell_own, cell_other = (a, mb), (a, pb)
                    else:
                        if stale is None:
                            raise NameError("name 'M_M_sub' is not defined")
                        own = stale[ii, jj].sum()
                        other = Mx[a - s:a + s + 1, pb - s:pb + s + 1][ii, jj].sum()
                        cell_own, cell_other = (a, mb), (a, pb)
                else:
                    b = p2 + P[hap + c1][0]
                    mb, pb = p1 + P["M" + c2][0], p1 + P["P" + c2][0]
                    if b < s or mb < s or pb < s or b + s + 1 > n or mb + s + 1 > n or pb + s + 1 > n:
                        continue
                    msub = Mx[mb - s:mb + s + 1, b - s:b + s + 1]
                    psub = Mx[pb - s:pb + s + 1, b - s:b + s + 1]
                    if hap == "M":
                        stale = msub
                        own, other = msub[ii, jj].sum(), psub[ii, jj].sum()
                        cell_own, cell_other = (b, mb), (b, pb)
                    else:
                        own, other = psub[ii, jj].sum(), msub[ii, jj].sum()
                        cell_own, cell_other = (pb, b), (mb, b)
                if own >= imin and (own / (own + other)) > iratio:
                    _inc(IW[res], *cell_own)
                elif other >= imin and (other / (own + other)) > iratio:
                    _inc(IW[res], *cell_other)
    return IW, IL


def _inc(M, i, j):
    if i >= M.shape[0] or j >= M.shape[1]:
        raise IndexError("index out of bounds")
    M[i][j] += 1
