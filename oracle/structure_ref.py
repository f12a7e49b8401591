"""ORACLE (test infrastructure only) — StructureFind numeric cores restated in
vectorised NumPy: compartment (distance decay, O/E, Pearson correlation,
top-3 PCA, PC selection) and the directionality-index TAD scan.

Pinned against golden vectors produced by the reference's own methods
(tests/golden/make_golden.py → tests/golden/compartment_*.npz, di_*.npz).

Deviation recorded in SURVEY.md §0.5 / §8(c): the reference's
``PCA(n_components=3)`` (StructureFind.py:338) uses randomized SVD for inputs
larger than 500×500; the oracle uses the exact SVD (``svd_solver='full'``).
"""
from __future__ import annotations

import numpy as np


# ---------------------------------------------------------------- compartment
def distance_decay(M, gap_ratio=0.05):
    """Distance_Decay (StructureFind.py:201-271) with ``G_array=None``.

    Gap columns: nonzero fraction <= 0.05.  decline[d] = sum of nonzero
    entries at |i-j| = d whose COLUMN is not a gap, divided by the number of
    valid pairs (2(size-d) - gaps, or size - |G| for d = 0) when positive.
    Returns (decline, G, NG)."""
    M = np.asarray(M, dtype=np.float64)
    size = M.shape[0]
    frac = (M != 0).sum(axis=0) / float(size)
    gmask = frac <= gap_ratio
    G = np.nonzero(gmask)[0]
    NG = np.nonzero(~gmask)[0]
    i, j = np.nonzero(M)
    keep = ~gmask[j]
    i, j = i[keep], j[keep]
    d = np.abs(j - i)
    decline = np.bincount(d, weights=M[i, j], minlength=size + 1).astype(np.float64)[:size + 1]
    dd = np.arange(size)
    n_lo = np.searchsorted(G, size - 1 - dd, side="right")     # #{g <= size-1-d}
    n_hi = G.size - np.searchsorted(G, dd, side="left")        # #{g >= d}
    bin_num = 2.0 * (size - dd) - (n_lo + n_hi)
    bin_num[0] = float(size) - G.size
    ok = bin_num > 0
    out = decline[:size].copy()
    out[ok] = out[ok] / bin_num[ok]
    return out, G, NG


def oe_matrix(M, decline):
    """O/E with the zero-decline fix (Get_PCA :323-329). Returns full N×N O/E."""
    M = np.asarray(M, dtype=np.float64)
    dec = np.array(decline, dtype=np.float64)
    dec[dec == 0] = dec[np.nonzero(dec)].min()
    N = M.shape[0]
    idx = np.arange(N)
    D = dec[np.abs(idx[:, None] - idx[None, :])]
    OE = np.zeros_like(M)
    nz = M != 0
    OE[nz] = M[nz] / D[nz]
    return OE


def sliding_oe(M, decline, step):
    """Sliding_Approach (StructureFind.py:274-299): inside
    [step, N-step-1]^2 the (2 step+1)^2 box sum of M over the 3-2-1 weighted
    expected sum of five diagonals; M / decline[|i-j|] on the border.
    ``decline`` already has the zero fix of Get_PCA :321.  Vectorised: box
    sums from a 2-D cumulative sum (rounding-level difference only)."""
    M = np.asarray(M, dtype=np.float64)
    dec = np.asarray(decline, dtype=np.float64)
    N = M.shape[0]
    if step < 1:
        raise IndexError("Sliding_Approach with step 0 reads decline[N]")
    idx = np.arange(N)
    dd = idx[:, None] - idx[None, :]
    OE = M / dec[np.abs(dd)]
    lo, hi = step, N - step - 1
    if hi >= lo:
        P = np.zeros((N + 1, N + 1))
        P[1:, 1:] = M.cumsum(0).cumsum(1)
        a = np.arange(lo, hi + 1)
        r0, r1 = a[:, None] - step, a[:, None] + step + 1
        c0, c1 = a[None, :] - step, a[None, :] + step + 1
        O = P[r1, c1] - P[r0, c1] - P[r1, c0] + P[r0, c0]
        d = dd[lo:hi + 1, lo:hi + 1]
        E = (3 * dec[np.abs(d)] + 2 * dec[np.abs(d - 1)] + 2 * dec[np.abs(d + 1)] + dec[np.abs(d - 2)]
             + dec[np.abs(d + 2)])
        OE[lo:hi + 1, lo:hi + 1] = O / E
    return OE


def pearson_columns(X):
    """np.corrcoef(X, rowvar=False) with NaN→0, inf→1 (Get_PCA :335-337)."""
    with np.errstate(invalid="ignore", divide="ignore"):
        C = np.corrcoef(X, rowvar=False)
    C = np.atleast_2d(C)
    C[np.isnan(C)] = 0
    C[np.isinf(C)] = 1
    return C


def top_components(C, k=3):
    """Top-k right singular vectors of the column-centred matrix — what
    ``PCA(n_components=k).fit(C).components_`` returns, exact SVD
    (Get_PCA :338-340).  Signs follow sklearn>=1.5 (max-|.| entry positive)."""
    X = C - C.mean(axis=0)
    _, _, Vt = np.linalg.svd(X, full_matrices=False)
    V = Vt[:k].copy()
    for r in range(V.shape[0]):
        if V[r, np.argmax(np.abs(V[r]))] < 0:
            V[r] = -V[r]
    return V


def top_components_eigsh(C, k=3):
    """The same components as ``top_components`` for large n, without a dense
    SVD: the top-k eigenvectors of A = Xc^T Xc (Xc = C - 1 mu^T, the matrix
    sklearn factors) by ARPACK (``scipy.sparse.linalg.eigsh``, tol 0 =
    machine precision) on matrix-vector products with C only; sklearn>=1.5
    signs.  Used where the exact SVD of n ~ 1e4 would take minutes (C5 chr1,
    VERDICT r3 item 4)."""
    from scipy.sparse.linalg import LinearOperator, eigsh
    C = np.asarray(C, dtype=np.float64)
    n = C.shape[1]
    mu = C.mean(axis=0)
    CT = C.T

    def mv(v):
        v = np.ravel(v)
        w = C @ v - (mu @ v)           # Xc v
        return CT @ w - mu * w.sum()   # Xc^T w

    A = LinearOperator((n, n), matvec=mv, dtype=np.float64)
    vals, vecs = eigsh(A, k=k, which="LA", tol=0, v0=np.ones(n) / np.sqrt(n), ncv=min(n, max(2 * k + 1, 24)))
    order = np.argsort(vals)[::-1]
    V = vecs[:, order].T.copy()
    for r in range(V.shape[0]):
        if V[r, np.argmax(np.abs(V[r]))] < 0:
            V[r] = -V[r]
    return V, vals[order]


def get_pca(decline, M, NG, SA=False, res=None, solver="svd"):
    """Get_PCA (StructureFind.py:302-342). Returns (pcs, Cor, OE[:, NG]);
    SA=True: Sliding_Approach with window 600 kb at resolution ``res``;
    ``solver="eigsh"``: components by top_components_eigsh (large n)."""
    if SA:
        dec = np.array(decline, dtype=np.float64)
        dec[dec == 0] = dec[np.nonzero(dec)].min()
        OE = sliding_oe(M, dec, 600000 // res // 2)[:, NG]
    else:
        OE = oe_matrix(M, decline)[:, NG]
    C = pearson_columns(OE)
    pcs = top_components(C, 3) if solver == "svd" else top_components_eigsh(C, 3)[0]
    return pcs, C, OE


def means_minus(C, pc, eps=1e-5):
    """Select_PC_new.means_minus (StructureFind.py:375-402)."""
    loc = np.arange(len(pc))
    a, b = pc > 0, pc < 0
    if not a.any() or not b.any():
        return 0
    la, lb = loc[a], loc[b]
    size_a = la.max() - la.min()
    size_b = lb.max() - lb.min()
    lens = max(la.max(), lb.max()) - min(la.min(), lb.min())
    Ca, Cb, Cab = C[a][:, a], C[b][:, b], C[a][:, b]
    va = Ca[(Ca > -1) & (Ca < 1 - eps)]
    vb = Cb[(Cb > -1) & (Cb < 1 - eps)]
    vab = Cab[(Cab > -1) & (Cab < 1)]
    same = np.concatenate([va, vb])
    if vab.size == 0 or vab.mean() == 0 or vab.mean() == -1 or size_a <= lens / 2 or size_b <= lens / 2:
        return 0
    return same.mean() - vab.mean()


def select_ab(OE, pc):
    """Select_PC_new.select_ab (:403-413): flip so that the A compartment has
    the larger mean nonzero O/E."""
    a, b = pc > 0, pc < 0
    A, B = OE[a][:, a], OE[b][:, b]
    va = A[A != 0].mean()
    vb = B[B != 0].mean()
    return pc.copy() * -1 if vb > va else pc


def select_pc(C, OE_ng, pcs):
    """Select_PC_new (:374-423). ``OE_ng`` = OE rows and columns at NG."""
    nums, values = 0, 0
    for i in range(len(pcs)):
        m = means_minus(C, pcs[i])
        if m > values:
            values, nums = m, i
    return select_ab(OE_ng, pcs[nums]), nums


def select_allelic_pc(pcs_full, trad_pc):
    """Select_Allelic_PC (:446-460): max |Pearson| with the traditional PC."""
    pcc = [abs(np.corrcoef(pc, trad_pc)[0][1]) for pc in pcs_full]
    return pcs_full[int(np.argmax(pcc))], int(np.argmax(pcc))


def compartment(M, solver="svd"):
    """Traditional compartment call for one chromosome (Compartment :509-527).
    Returns (pc_full[N], selected_index, pcs, Cor)."""
    dec, G, NG = distance_decay(M)
    pcs, C, OE = get_pca(dec, M, NG, solver=solver)
    pc, k = select_pc(C, OE[NG], pcs)
    out = np.zeros(M.shape[0])
    out[NG] = pc
    return out, k, pcs, C


def refill_gap(M1, M2, NonGap, dtype):
    """Refill_Gap (StructureFind.py:463-488), loop for loop -- including the
    transpose inside the 'OE' loop (:483-486)."""
    R = np.zeros(np.shape(M1), dtype=float)
    if dtype == "Cor":
        tmp = np.zeros((np.shape(M1)[0], np.shape(M2)[0]), dtype=float)
        for i in range(len(NonGap)):
            tmp[NonGap[i]] = M2[i]
        tmp = tmp.T
        for i in range(len(NonGap)):
            R[NonGap[i]] = tmp[i]
    elif dtype == "OE":
        M2 = np.asarray(M2).T
        for i in range(len(NonGap)):
            R[NonGap[i]] = M2[i]
            R = R.T
    return R


# ------------------------------------------------------------------- TAD / DI
def get_gap(M, min_tad, res):
    """Get_Gap (StructureFind.py:721-751) plus the first/last-bin rule of
    Data_preprocess (:875-883). Returns sorted int64 gap indices."""
    M = np.asarray(M)
    N = M.shape[0]
    lb = int(min_tad / res)
    t = 2 * lb * 0.8
    gap = np.ones(N, dtype=bool)
    for i in range(lb, N - lb):
        gap[i] = np.count_nonzero(M[i - lb:i + lb, i]) < t
    gap[0] = True
    gap[N - 1] = True
    return np.nonzero(gap)[0].astype(np.int64)


def get_di(M, gap, w, test_type="ttest"):
    """Get_DI (StructureFind.py:804-839) with a constant window ``w`` bins."""
    M = np.asarray(M, dtype=np.float64)
    N = M.shape[0]
    g = np.zeros(N, dtype=bool)
    g[np.asarray(gap, dtype=np.int64)] = True
    DI = np.zeros(N)
    for j in range(N):
        if g[j] or j < w or j > N - w - 1:
            continue
        up = M[j - w:j, j][::-1]
        down = M[j + 1:j + w + 1, j]
        val = 0.0
        if test_type == "ttest":
            um, dm = up.mean(), down.mean()
            ud = np.sum((up - um) ** 2 / (up.size * (up.size - 1)))
            dd = np.sum((down - dm) ** 2 / (down.size * (down.size - 1)))
            den = np.sqrt(ud + dd)
            if den != 0:
                val = (dm - um) / den
        else:
            us, ds = up.sum(), down.sum()
            e = float(us + ds) / 2.0
            if us != ds and e != 0:
                val = float(ds - us) / abs(ds - us) * ((us - e) ** 2 / e + (ds - e) ** 2 / e)
        DI[j] = val
    return DI


# ----------------------------------------------- banded restatement (large N)
def band_from_pixels(bin1, bin2, count, weight, lo, N, B):
    """Diagonal-major band of one chromosome's balanced matrix from cooler's
    pixel table: band[B + k, j] = M[j + k, j] for |k| <= B, M = count * w[bin1]
    * w[bin2] with NaN -> 0 (Data_preprocess :853-854; weight None = raw)."""
    b1 = np.asarray(bin1, dtype=np.int64) - lo
    b2 = np.asarray(bin2, dtype=np.int64) - lo
    v = np.asarray(count, dtype=np.float64)
    sel = (b1 >= 0) & (b2 < N) & (np.abs(b2 - b1) <= B)
    i, j, v = b1[sel], b2[sel], v[sel]
    if weight is not None:
        w = np.asarray(weight, dtype=np.float64)
        v = v * w[i + lo] * w[j + lo]
        v[np.isnan(v)] = 0.0
    band = np.zeros((2 * B + 1, N))
    d = j - i
    band[B - d, j] = v      # M[i][j] = M[j - d][j]
    band[B + d, i] = v      # M[j][i] = M[i + d][i]
    return band


def get_gap_band(band, B, lb):
    """Get_Gap (StructureFind.py:721-751) on the band, plus the first / last
    bin (Data_preprocess :875-883): column i is a gap when fewer than
    2 lb 0.8 of M[i - lb : i + lb, i] are nonzero, or within lb of an edge."""
    N = band.shape[1]
    nz = np.zeros(N, dtype=np.int64)
    for k in range(-lb, lb):
        nz += band[B + k] != 0
    gap = np.ones(N, dtype=bool)
    inner = np.arange(lb, N - lb)
    gap[inner] = nz[inner] < 2 * lb * 0.8
    gap[0] = gap[N - 1] = True
    return np.nonzero(gap)[0].astype(np.int64)


def get_di_band(band, B, gap, w, test_type="ttest"):
    """Get_DI (StructureFind.py:804-839) on the band: up = M[j-w:j, j] reversed
    (band rows B-1 .. B-w), down = M[j+1:j+w+1, j] (rows B+1 .. B+w); the same
    per-column arithmetic as get_di."""
    N = band.shape[1]
    g = np.zeros(N, dtype=bool)
    g[np.asarray(gap, dtype=np.int64)] = True
    DI = np.zeros(N)
    for j in range(N):
        if g[j] or j < w or j > N - w - 1:
            continue
        up = band[B - 1:B - w - 1:-1, j] if B - w - 1 >= 0 else band[B - 1::-1, j][:w]
        down = band[B + 1:B + w + 1, j]
        val = 0.0
        if test_type == "ttest":
            um, dm = up.mean(), down.mean()
            ud = np.sum((up - um) ** 2 / (up.size * (up.size - 1)))
            dd = np.sum((down - dm) ** 2 / (down.size * (down.size - 1)))
            den = np.sqrt(ud + dd)
            if den != 0:
                val = (dm - um) / den
        else:
            us, ds = up.sum(), down.sum()
            e = float(us + ds) / 2.0
            if us != ds and e != 0:
                val = float(ds - us) / abs(ds - us) * ((us - e) ** 2 / e + (ds - e) ** 2 / e)
        DI[j] = val
    return DI
