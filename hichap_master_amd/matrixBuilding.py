"""HiCHap's diploid bias correction on MI355X — same entry points as
``HiCHap/matrixBuilding.py``.

* ``TwoStepCorrection(TM, MM, PM)``            matrixBuilding.py:984-1023
* ``IntraChromMatrixCorrection(Tra, Hap)``     matrixBuilding.py:1026-1041
* ``GenomeWideMatrixCorrection(Bins_Pos, Hap_Bins_Pos, T_M, H_M)``  :857-901
* ``Sort_Chromosomes(chro_lst)``               :388-406

Every O(N^2) step runs in HIP kernels (``hh_dense_rowstats``: row sums and
zero counts; ``hh_dense_symvc``: gap-aware symmetrisation + VC^(2/3) + mean
rescale, fused).  What stays on the host is O(N) glue on per-row vectors,
written with the same NumPy calls as the reference so the gap and alpha
decisions are bit-identical (``np.percentile`` linear interpolation, the
``max``/``==0`` fix-ups, true division of exact integer row sums).
"""
from __future__ import annotations

import ctypes as C
import json
import os

import numpy as np

from . import _lib
from ._lib import call, ptr

VC_EXPONENT = 2 / 3  # Correct_VC(X, 2/3) under `from __future__ import division` (:8, :1014)


# ------------------------------------------------------------------ kernels
def _as_dense(X):
    X = np.asarray(X)
    if X.ndim != 2 or X.shape[0] != X.shape[1]:
        raise ValueError("expected a square matrix")
    if np.issubdtype(X.dtype, np.integer) or X.dtype == np.bool_:
        return np.ascontiguousarray(X, dtype=np.int64), 0
    return np.ascontiguousarray(X, dtype=np.float64), 1


def row_stats(X, lo=None, hi=None, stream=None):
    """Per-row (sum, zero count) over columns [lo_i, hi_i) on the GPU."""
    _lib.require_gpu()
    A, dt = _as_dense(X)
    N = A.shape[0]
    s = np.empty(N, np.float64)
    z = np.empty(N, np.int64)
    l = None if lo is None else np.ascontiguousarray(lo, dtype=np.int64)
    h = None if hi is None else np.ascontiguousarray(hi, dtype=np.int64)
    call("hh_dense_rowstats", ptr(A), dt, N, ptr(l), ptr(h), ptr(s), ptr(z), 0, stream)
    return s, z


def sym_vc_rescale(X, alpha, gap_idx, raw_sum, exponent=VC_EXPONENT, stream=None):
    """(mean(X)/mean(C)) * C, C = Correct_VC(Trans2symmetry(X/alpha[:,None], gap), exponent).
    ``gap_idx`` None -> the sum form (no gap / Trans2symmetryLowRes)."""
    _lib.require_gpu()
    A, dt = _as_dense(X)
    N = A.shape[0]
    a = np.ascontiguousarray(alpha, dtype=np.float64)
    g = None
    if gap_idx is not None:
        g = np.zeros(N, np.uint8)
        g[np.asarray(gap_idx, dtype=np.int64)] = 1
    out = np.empty((N, N), np.float64)
    call("hh_dense_symvc", ptr(A), dt, N, ptr(a), ptr(g), float(exponent), float(raw_sum), ptr(out), 0, stream)
    return out


# --------------------------------------------------------------- host glue
def _coverage(zeros, n):
    """Coverage_M (:904-912): 1 - zeros / float(len(row))."""
    return 1 - (np.asarray(zeros) / float(n))


def _gap_from_coverage(cov):
    """Gap_defined (:915-929) given the coverage vector."""
    threshold = np.percentile(cov[np.nonzero(cov)], 25)
    if threshold > 0.2:
        threshold = 0.2
    return np.nonzero(cov < threshold)[0].astype(np.int64)


def _non_gap(N, gap):
    """Non_Gap_Defined (:932-942)."""
    keep = np.ones(N, dtype=bool)
    keep[np.asarray(gap, dtype=np.int64)] = False
    return np.nonzero(keep)[0]


def _snp_alpha(m_sum, p_sum, t_sum, non_gap):
    """SNP-density factor (:994-1005 / :878-886) on exact integer row sums."""
    alpha = (m_sum + p_sum) / (t_sum + 1)
    alpha /= np.max(alpha[non_gap])
    alpha[alpha == 0] = 1
    threshold = np.percentile(alpha[non_gap], 20)
    alpha[alpha < threshold] = threshold
    return alpha


# ------------------------------------------------------------------- API
def TwoStepCorrection(TM, MM, PM):
    """Two-step correction of one chromosome's maternal / paternal matrices
    (matrixBuilding.py:984-1023).  Returns (Nor_MM, Nor_PM, Gap_M, Gap_P).

    One C-ABI call (``hh_twostep``): each matrix is uploaded once, the gap /
    alpha glue runs in C++ with np.percentile semantics."""
    _lib.require_gpu()
    on_dev = [bool(getattr(X, "is_cuda", False)) for X in (TM, MM, PM)]
    if all(on_dev):
        return _twostep_device(TM, MM, PM)
    if any(on_dev):
        raise ValueError("TM, MM, PM must all be device tensors or all host arrays")
    # host arrays (NumPy, or CPU torch tensors: np.asarray takes them as is)
    mats = [np.ascontiguousarray(np.asarray(X), dtype=np.int64) for X in (TM, MM, PM)]
    N = mats[0].shape[0]
    if any(X.ndim != 2 or X.shape != (N, N) for X in mats):
        raise ValueError("TM, MM, PM must be square matrices of the same size")
    Nor_MM = np.empty((N, N), np.float64)
    Nor_PM = np.empty((N, N), np.float64)
    gm = np.empty(N, np.uint8)
    gp = np.empty(N, np.uint8)
    call("hh_twostep", ptr(mats[0]), ptr(mats[1]), ptr(mats[2]), N, ptr(Nor_MM), ptr(Nor_PM), ptr(gm), ptr(gp), 0,
         None)
    return Nor_MM, Nor_PM, np.nonzero(gm)[0].astype(np.int64), np.nonzero(gp)[0].astype(np.int64)


def _twostep_device(TM, MM, PM, stream=None):
    """TwoStepCorrection on int64 device tensors: no host round trip; returns
    (Nor_MM, Nor_PM) as float64 device tensors and the gap index arrays."""
    import torch
    N = int(TM.shape[0])
    for X in (TM, MM, PM):
        if tuple(X.shape) != (N, N) or X.dtype != torch.int64 or not X.is_cuda or not X.is_contiguous():
            raise ValueError("TM, MM, PM must be contiguous int64 N x N device tensors")
    nm = torch.empty((N, N), dtype=torch.float64, device=TM.device)
    npm = torch.empty((N, N), dtype=torch.float64, device=TM.device)
    gm = np.empty(N, np.uint8)
    gp = np.empty(N, np.uint8)
    dp = lambda t: C.c_void_p(t.data_ptr())
    call("hh_twostep", dp(TM), dp(MM), dp(PM), N, dp(nm), dp(npm), ptr(gm), ptr(gp), 1, stream)
    return nm, npm, np.nonzero(gm)[0].astype(np.int64), np.nonzero(gp)[0].astype(np.int64)


def dense_from_cells_device(cells, N, offset=0, symmetric=False, stream=None):
    """Dense int64 N x N device tensor from (row, col, count) cells (host
    arrays or int64 device tensors) -- the reference's dense matrices
    (:554, :567-570, :1290-1301) built on the GPU so only cells cross PCIe.
    ``symmetric``: an upper-triangle table mirrored (T); else ordered cells
    (the asymmetric imputed MM / PM)."""
    import torch
    out = torch.empty((int(N), int(N)), dtype=torch.int64, device="cuda")
    on_dev = hasattr(cells[0], "data_ptr")
    if on_dev:
        arrs = [x.to(torch.int64).contiguous() for x in cells]
        ps = [C.c_void_p(x.data_ptr()) for x in arrs]
        n = int(arrs[0].numel())
    else:
        arrs = [np.ascontiguousarray(x, dtype=np.int64) for x in cells]
        ps = [ptr(x) for x in arrs]
        n = int(arrs[0].size)
    call("hh_dense_from_cells", ps[0], ps[1], ps[2], n, int(N), int(offset), int(bool(symmetric)), int(on_dev),
         C.c_void_p(out.data_ptr()), stream)
    return out


def upper_table_device(X, stream=None):
    """np.triu(X).nonzero() of a dense fp64 device matrix as (bin1, bin2,
    value) int32 / int32 / float64 device tensors in cooler order -- what
    NPZ2Cooler writes for a corrected matrix (:1613, :1628-1633)."""
    import torch
    N = int(X.shape[0])
    m = C.c_int64(0)
    call("hh_dense_upper_count", C.c_void_p(X.data_ptr()), N, C.byref(m), stream)
    out = [torch.empty(max(int(m.value), 1), dtype=dt, device=X.device)
           for dt in (torch.int32, torch.int32, torch.float64)]
    call("hh_dense_upper_write", C.c_void_p(X.data_ptr()), N, *(C.c_void_p(t.data_ptr()) for t in out), stream)
    return tuple(t[:int(m.value)] for t in out)


def TwoStepCorrectionPixels(N, T_pixels, MM_cells, PM_cells, offset=0, output="upper", stream=None):
    """TwoStepCorrection (:984-1023) fed by the tables the matrix
    construction produces -- T as an upper-triangle pixel table, the imputed
    MM / PM as ordered cells (asymmetric, :1290-1301) -- with the dense
    matrices built and corrected on the GPU: only the cells cross PCIe, not
    3 x N^2 x 8 B in and 2 x N^2 x 8 B out.  ``output="upper"``: the
    corrected matrices' upper-triangle tables (bin1, bin2, value) as host
    arrays -- the triu COO NPZ2Cooler stores (:1613, :1628-1633);
    ``"device"``: dense float64 device tensors.  Returns (Nor_MM, Nor_PM,
    Gap_M, Gap_P)."""
    _lib.require_gpu()
    TM = dense_from_cells_device(T_pixels, N, offset, True, stream)
    MM = dense_from_cells_device(MM_cells, N, offset, False, stream)
    PM = dense_from_cells_device(PM_cells, N, offset, False, stream)
    nm, npm, gm, gp = _twostep_device(TM, MM, PM, stream)
    del TM, MM, PM
    if output == "device":
        return nm, npm, gm, gp
    if output != "upper":
        raise ValueError("output must be 'upper' or 'device'")
    res = []
    for X in (nm, npm):
        b1, b2, v = upper_table_device(X, stream)
        res.append((b1.cpu().numpy().astype(np.int64) + offset, b2.cpu().numpy().astype(np.int64) + offset,
                    v.cpu().numpy()))
    return res[0], res[1], gm, gp


TWOSTEP_STREAMS = 0  # hh_twostep_batch: 0 = every pass of every chromosome in one shared launch


def IntraChromMatrixCorrection(Tra_Lib, Hap_Lib, n_streams=TWOSTEP_STREAMS, stream=None):
    """Per-chromosome TwoStepCorrection (matrixBuilding.py:1026-1041).  With
    device tensors, every chromosome in one ``hh_twostep_batch`` call (shared
    launches per pass, or with ``n_streams`` > 0 the chains on that many
    streams; outputs device tensors)."""
    keys = list(Tra_Lib.keys())
    mats = [(Tra_Lib[c], Hap_Lib["M" + c], Hap_Lib["P" + c]) for c in keys]
    if mats and all(bool(getattr(X, "is_cuda", False)) for t in mats for X in t):
        return _intra_batch_device(keys, mats, n_streams, stream)
    Nor_Lib, Gap_Lib = {}, {}
    for chro in Tra_Lib.keys():
        Nor_MM, Nor_PM, Gap_M, Gap_P = TwoStepCorrection(Tra_Lib[chro], Hap_Lib["M" + chro], Hap_Lib["P" + chro])
        Nor_Lib["M" + chro] = Nor_MM
        Nor_Lib["P" + chro] = Nor_PM
        Gap_Lib["M" + chro] = Gap_M
        Gap_Lib["P" + chro] = Gap_P
    return Nor_Lib, Gap_Lib


def _intra_batch_device(keys, mats, n_streams, stream=None):
    import torch
    _lib.require_gpu()
    Ns = []
    for T, M, P in mats:
        N = int(T.shape[0])
        for X in (T, M, P):
            if tuple(X.shape) != (N, N) or X.dtype != torch.int64 or not X.is_contiguous():
                raise ValueError("TM, MM, PM must be contiguous int64 N x N device tensors")
        Ns.append(N)
    nm = [torch.empty((N, N), dtype=torch.float64, device=mats[0][0].device) for N in Ns]
    npm = [torch.empty((N, N), dtype=torch.float64, device=mats[0][0].device) for N in Ns]
    n = len(keys)
    arr = lambda xs: (C.c_void_p * n)(*[C.c_void_p(x.data_ptr()) for x in xs])
    Narr = np.asarray(Ns, dtype=np.int64)
    gm = np.empty(int(Narr.sum()), np.uint8)
    gp = np.empty(int(Narr.sum()), np.uint8)
    call("hh_twostep_batch", n, arr([t[0] for t in mats]), arr([t[1] for t in mats]), arr([t[2] for t in mats]),
         ptr(Narr), arr(nm), arr(npm), ptr(gm), ptr(gp), int(n_streams), stream)
    off = np.concatenate([[0], np.cumsum(Narr)])
    Nor_Lib, Gap_Lib = {}, {}
    for k, c in enumerate(keys):
        Nor_Lib["M" + c], Nor_Lib["P" + c] = nm[k], npm[k]
        Gap_Lib["M" + c] = np.nonzero(gm[off[k]:off[k + 1]])[0].astype(np.int64)
        Gap_Lib["P" + c] = np.nonzero(gp[off[k]:off[k + 1]])[0].astype(np.int64)
    return Nor_Lib, Gap_Lib


def Sort_Chromosomes(chro_lst):
    """Numeric labels ascending, then the rest sorted; leading 'c','h','r'
    characters stripped as the reference's ``lstrip('chr')`` does (:388-406)."""
    names = [i.lstrip("chr") for i in chro_lst]
    num, txt = [], []
    for i in names:
        try:
            num.append(int(i))
        except ValueError:
            txt.append(i)
    return [str(j) for j in sorted(num)] + sorted(txt)


def GenomeWideMatrixCorrection(Bins_Pos, Hap_Bins_Pos, T_M, H_M):
    """Whole-genome diploid correction (matrixBuilding.py:857-901).

    ``Bins_Pos[c] = (start, end)`` inclusive bin ranges of T_M;
    ``Hap_Bins_Pos['M'+c]`` / ``['P'+c]`` the same in H_M (2n x 2n)."""
    T_M = np.asarray(T_M)
    H_M = np.asarray(H_M)
    n, n2 = T_M.shape[0], H_M.shape[0]
    t_lo, t_hi = np.zeros(n, np.int64), np.full(n, n, np.int64)
    h_lo, h_hi = np.zeros(n2, np.int64), np.full(n2, n2, np.int64)
    for c, (s, e) in Bins_Pos.items():
        t_lo[s:e + 1], t_hi[s:e + 1] = s, e + 1
        for h in ("M", "P"):
            hs, he = Hap_Bins_Pos[h + c]
            h_lo[hs:he + 1], h_hi[hs:he + 1] = hs, he + 1
    t_sum, t_zero = row_stats(T_M, t_lo, t_hi)       # block-restricted (Tra_M = T_M[s:e+1, s:e+1])
    h_sum, _ = row_stats(H_M, h_lo, h_hi)            # M_M / P_P diagonal blocks
    h_full, _ = row_stats(H_M)                       # H_M.mean()
    Beta = {}
    for chro in Bins_Pos.keys():
        s, e = Bins_Pos[chro]
        ms, me = Hap_Bins_Pos["M" + chro]
        ps, pe = Hap_Bins_Pos["P" + chro]
        L = e - s + 1
        cov = _coverage(t_zero[s:e + 1], L)
        gap = np.nonzero(cov < 0.1)[0]              # Gap_definedLowRes (:742-753)
        non_gap = _non_gap(L, gap)
        Beta[chro] = _snp_alpha(h_sum[ms:me + 1], h_sum[ps:pe + 1], t_sum[s:e + 1], non_gap)
    Alpha = np.concatenate([Beta[i] for i in Sort_Chromosomes(list(Beta.keys()))]).astype(np.float64)
    return sym_vc_rescale(H_M, np.concatenate([Alpha, Alpha]), None, h_full.sum())


def _gw_layout(Bins_Pos, Hap_Bins_Pos):
    """chrom_offsets of T's layout (chromosomes in bin order) and a check that
    H is the M copies then the P copies of the same layout (:429-454)."""
    items = sorted(Bins_Pos.items(), key=lambda kv: kv[1][0])
    off = [0]
    for c, (s, e) in items:
        if s != off[-1]:
            raise ValueError("Bins_Pos must tile [0, n) contiguously")
        off.append(e + 1)
    n = off[-1]
    for c, (s, e) in items:
        if tuple(Hap_Bins_Pos["M" + c]) != (s, e) or tuple(Hap_Bins_Pos["P" + c]) != (n + s, n + e):
            raise ValueError("Hap_Bins_Pos must be the M copies then the P copies of Bins_Pos' layout")
    return np.asarray(off, dtype=np.int64), [c for c, _ in items]


def GenomeWideMatrixCorrectionSparse(Bins_Pos, Hap_Bins_Pos, T_pixels, H_cells, exponent=VC_EXPONENT,
                                     stream=None, device_result=False, numpy_alpha=False):
    """GenomeWideMatrixCorrection (matrixBuilding.py:857-901) on pixel tables:
    the whole-genome diploid matrices at 10 kb are 607 282 x 607 282, which the
    reference's dense form cannot hold.

    ``T_pixels`` = (bin1, bin2, count): cooler's upper-triangle table of T_M
    (sorted by (bin1, bin2)); ``H_cells`` = (row, col, count): every nonzero
    cell of the asymmetric imputed H_M (sorted by (row, col)).  Either may be
    host arrays or int32 device tensors (then both must be).  Returns the
    upper triangle of the corrected matrix as (bin1, bin2, value), cooler
    order — the table NPZ2Cooler writes for it (:1613, :1628-1633).  The alpha
    step (:878-893) uses the reference's NumPy expressions on exact integer
    row sums computed on the GPU: in C++ overlapped with the column-list
    build (hh_gw_alpha), or here with NumPy (numpy_alpha=True; the same
    bits, tests/test_gw_sparse_gpu.py)."""
    _lib.require_gpu()
    import os
    import time
    tick = [time.perf_counter()]
    timing = os.environ.get("HH_GW_TIMING")

    def lap(what):  # HH_GW_TIMING=1: host-side phase times (diagnostic)
        if timing:
            t = time.perf_counter()
            print(f"[gw] {what}: {1e3 * (t - tick[0]):.2f} ms", flush=True)
            tick[0] = t
    off, order = _gw_layout(Bins_Pos, Hap_Bins_Pos)
    n = int(off[-1])
    h = C.c_void_p()
    on_dev = hasattr(H_cells[0], "data_ptr")
    if on_dev:
        def dp(x):
            return C.c_void_p(x.data_ptr())
        call("hh_gw_create_device", dp(T_pixels[0]), dp(T_pixels[1]), dp(T_pixels[2]), int(T_pixels[0].numel()),
             dp(H_cells[0]), dp(H_cells[1]), dp(H_cells[2]), int(H_cells[0].numel()), n, ptr(off), len(order),
             stream, C.byref(h))
    else:
        t = [np.ascontiguousarray(x, dtype=dt) for x, dt in zip(T_pixels, (np.int64, np.int64, np.float64))]
        hc = [np.ascontiguousarray(x, dtype=dt) for x, dt in zip(H_cells, (np.int64, np.int64, np.float64))]
        call("hh_gw_create", ptr(t[0]), ptr(t[1]), ptr(t[2]), t[0].size, ptr(hc[0]), ptr(hc[1]), ptr(hc[2]),
             hc[0].size, n, ptr(off), len(order), stream, C.byref(h))
    lap("create")
    try:
        # the alpha step: computed by hh_gw_create on a host thread while the
        # GPU built the column lists (the same NumPy operations in C++); a
        # chromosome it leaves (no non-gap bin, a max that is not positive
        # finite) takes the NumPy expressions below, as does numpy_alpha=True
        a_bins = np.empty(n, np.float64)
        ok = np.zeros(len(order), np.int32)
        if not numpy_alpha:
            call("hh_gw_alpha", h, ptr(a_bins), ptr(ok))
        stats = None
        Beta = {}
        for k, c in enumerate(order):
            s, e = Bins_Pos[c]
            if ok[k]:
                Beta[c] = a_bins[s:e + 1]
                continue
            if stats is None:
                t_sum = np.empty(n, np.int64)
                t_nz = np.empty(n, np.int64)
                h_bs = np.empty(2 * n, np.int64)
                h_tot = C.c_int64(0)
                call("hh_gw_stats", h, ptr(t_sum), ptr(t_nz), ptr(h_bs), C.byref(h_tot))
                stats = True
            L = e - s + 1
            cov = _coverage(L - t_nz[s:e + 1], L)
            gap = np.nonzero(cov < 0.1)[0]              # Gap_definedLowRes (:742-753)
            Beta[c] = _snp_alpha(h_bs[s:e + 1], h_bs[n + s:n + e + 1], t_sum[s:e + 1], _non_gap(L, gap))
        # the reference's list extend + `Alpha += Alpha` (:887-890) as one
        # concatenate: the same values without 600 k boxed floats (40 ms)
        Alpha = np.concatenate([Beta[i] for i in Sort_Chromosomes(list(Beta.keys()))]).astype(np.float64)
        Alpha = np.ascontiguousarray(np.concatenate([Alpha, Alpha]))
        lap("alpha")
        m = C.c_int64(0)
        if device_result:  # int32 / int32 / float64 device tensors, written in place by the library
            import torch
            call("hh_gw_correct_count", h, ptr(Alpha), float(exponent), C.byref(m), stream)
            lap("correct_count")
            m = int(m.value)
            out = [torch.empty(max(m, 1), dtype=dt, device="cuda") for dt in (torch.int32, torch.int32, torch.float64)]
            lap("outputs")
            call("hh_gw_correct_write", h, *(C.c_void_p(t.data_ptr()) for t in out), stream)
            lap("correct_write")
            return tuple(t[:m] for t in out)
        call("hh_gw_correct", h, ptr(Alpha), float(exponent), C.byref(m), stream)
        m = int(m.value)
        b1 = np.empty(m, np.int64)
        b2 = np.empty(m, np.int64)
        v = np.empty(m, np.float64)
        call("hh_gw_result", h, ptr(b1), ptr(b2), ptr(v), stream)
        return b1, b2, v
    finally:
        call("hh_gw_free", h)
        lap("free")


# ---------------------------------------------------------- pair binning
# Same entry points as the reference's matrix construction; the per-line
# loops run on the GPU (hichap_master_amd.pairs, csrc/pairs.hip).
def Load_Genome(genomeSize, chroms):
    """{stripped chrom: length} for the chromosomes `chroms` accepts (:349-366)."""
    from . import pairs
    return pairs.load_genome(genomeSize, chroms)


def Load_HaplotypeGenome(genomeSize, chroms):
    """{'M'+c: l, 'P'+c: l} (:369-385)."""
    g = Load_Genome(genomeSize, chroms)
    out = {}
    for c, l in g.items():
        out["M" + c] = l
        out["P" + c] = l
    return out


def Get_Chro_Bins(genomeSize, Resolution, chroms):
    """({chrom: (first, last)} inclusive, n_bins) (:409-426)."""
    from . import pairs
    return pairs.chrom_bins(Load_Genome(genomeSize, chroms), Resolution)


def Get_Chro_Bins_Haplotypes(genomeSize, Resolution, chroms):
    """M chromosomes then P chromosomes (:429-454)."""
    from . import pairs
    return pairs.haplotype_bins(Load_Genome(genomeSize, chroms), Resolution)


def _bin_sources(genome, chroms, passes, wholeRes, localRes, haplotype, local_halves):
    """Run the GPU binner over `passes` = [(source, PairsFormat)], one whole
    target per wholeRes and one intra-chromosome target per localRes."""
    from . import pairs
    B = pairs.PairBinner(genome, chroms)
    try:
        whole = {res: B.add_target(res, local=False, haplotype=haplotype) for res in wholeRes}
        local = {res: B.add_target(res, local=True, haplotype=haplotype) for res in localRes}
        for src, fmt in passes:
            B.feed(src, fmt)
        B.finish()
        wp = {res: B.pixels(t) for res, t in whole.items()}
        lp = {res: B.pixels(t) for res, t in local.items()}
        return B.order, whole, local, wp, lp
    finally:
        B.close()


def TraditionalMatrixBuilding(bed_IO, genomeSize, wholeRes, localRes, chroms):
    """Traditional matrices from *_Valid.bed pairs (:528-614).

    ``bed_IO``: a path, a list of paths (concatenated like `cat`), bytes, a
    file object or an iterable of lines.  Returns ``(Whole_Lib, Local_Lib)``
    in the reference's shape: ``Whole_Lib[res]`` = {chrom: upper-triangle
    sparse, 'c1_c2': inter block sparse}, ``Local_Lib[res]`` = {chrom:
    upper-triangle sparse}; sparse = structured (bin1, bin2, IF) arrays in
    chromosome-local bins (WholeMatrixToSparseDict / IntraMatrixToSparseDict,
    :457-525)."""
    from . import pairs
    genome = Load_Genome(genomeSize, chroms)
    fmt = pairs.pairs_format(pairs.VALID_BED)
    order, whole, local, wp, lp = _bin_sources(genome, chroms, [(bed_IO, fmt)], wholeRes, localRes, False, None)
    Whole_Lib, Local_Lib = {}, {}
    for res in wholeRes:
        bins, _ = pairs.chrom_bins(genome, res)
        Whole_Lib[res] = pairs.whole_sparse_dict(*wp[res], bins)
    for res in localRes:
        Local_Lib[res] = pairs.local_sparse_dict(*lp[res], local[res], order)
    return Whole_Lib, Local_Lib


def TraditionalMatrixInAllelic(bed_IO, genomeSize, wholeRes, localRes, chroms, dense=True):
    """Traditional matrices of the haplotype pipeline from the allelic beds
    (fields 0-3, no mark filter; :793-854).  Reference shape (dense=True):
    ``Whole_Lib[res] = {'Bins': Bins, 'Matrix': int64 n x n}``,
    ``Local_Lib[res][chrom]`` int64 N x N.  dense=False returns pixel tables
    ``(bin1, bin2, count)`` (global bins for whole, local bins per chrom)."""
    from . import pairs
    genome = Load_Genome(genomeSize, chroms)
    fmt = pairs.pairs_format(pairs.ALLELIC_BED)
    order, whole, local, wp, lp = _bin_sources(genome, chroms, [(bed_IO, fmt)], wholeRes, localRes, False, None)
    return _dense_libs(genome, order, whole, local, wp, lp, dense, haplotype=False)


def _dense_libs(genome, order, whole, local, wp, lp, dense, haplotype):
    from . import pairs
    Whole_Lib, Local_Lib = {}, {}
    for res, t in whole.items():
        bins, total = (pairs.haplotype_bins if haplotype else pairs.chrom_bins)(genome, res)
        b1, b2, c = wp[res]
        Whole_Lib[res] = {"Bins": bins,
                          "Matrix": pairs.dense_from_pixels(b1, b2, c, total) if dense else (b1, b2, c)}
    for res, t in local.items():
        b1, b2, c = lp[res]
        b1 = np.asarray(b1, np.int64)
        Local_Lib[res] = {}
        halves = ("M", "P") if haplotype else ("",)
        for h, prefix in enumerate(halves):
            for k, chro in enumerate(order):
                s0 = int(t.chrom_first[k]) + h * int(t.chrom_nbins.sum())
                n = int(t.chrom_nbins[k])
                lo, hi = np.searchsorted(b1, [s0, s0 + n], "left")
                if dense:
                    Local_Lib[res][prefix + chro] = pairs.dense_from_pixels(b1[lo:hi], b2[lo:hi], c[lo:hi], n, s0)
                else:
                    Local_Lib[res][prefix + chro] = (b1[lo:hi] - s0, np.asarray(b2[lo:hi], np.int64) - s0, c[lo:hi])
    return Whole_Lib, Local_Lib


def HaplotypeUnImputedBuilding(M_M, P_P, M_P, P_M, genomeSize, wholeRes, localRes, chroms, dense=True):
    """The unimputed haplotype matrices of HaplotypeMatrixBuilding
    (:1108-1240): M_M and P_P pairs with last field 'Both' (cis pairs also go
    to the per-haplotype intra-chromosome matrices), M_P pairs as (M chrom1,
    P chrom2) and P_M pairs as (P chrom1, M chrom2) in the 2n-bin whole-genome
    layout.  Each argument is a pair source (path, list of paths, bytes, ...).
    Returns ``(UnImputated_Whole_Lib, UnImputated_Local_Lib)`` in the
    reference's dense shape (``Local_Lib[res]['M'+c]``, ``['P'+c]``)."""
    from . import pairs
    genome = Load_Genome(genomeSize, chroms)
    passes = [(M_M, pairs.pairs_format(pairs.ALLELIC_BED, "Both", 0, 0)),
              (P_P, pairs.pairs_format(pairs.ALLELIC_BED, "Both", 1, 1)),
              (M_P, pairs.pairs_format(pairs.ALLELIC_BED, "", 0, 1)),
              (P_M, pairs.pairs_format(pairs.ALLELIC_BED, "", 1, 0))]
    order, whole, local, wp, lp = _bin_sources(genome, chroms, passes, wholeRes, localRes, True, None)
    return _dense_libs(genome, order, whole, local, wp, lp, dense, haplotype=True)


def _materialise(source):
    """Paths stay paths (read in blocks, seekable); anything else -> bytes."""
    import os
    if isinstance(source, (bytes, bytearray, memoryview, str, os.PathLike)):
        return source
    if isinstance(source, (list, tuple)) and source and all(isinstance(x, (str, os.PathLike)) and os.path.isfile(x)
                                                            for x in source):
        return list(source)
    from . import pairs
    return b"".join(pairs._iter_blocks(source, pairs.CHUNK_BYTES))


def HaplotypeImputation(M_M, P_P, genomeSize, wholeRes, localRes, chroms, Imputation_region, Imputation_min,
                        Imputation_ratio, UnImputated_Whole_Lib, UnImputated_Local_Lib):
    """The imputation passes of HaplotypeMatrixBuilding (:1251-1494) on the
    GPU: single-allele ('R1' / 'R2') lines of the M_M then P_P beds; intra-
    chromosome ones add an ordered count, inter-chromosome ones are imputed
    to the M or P copy whose neighbourhood (GetNeighborhoodIndex disc) in the
    unimputed whole matrix dominates.  The reference's quirks are kept: R2
    lines take chrom1's offset for pos2 (:1347-1349); the P pass's R1 branch
    sums the stale M_M_sub of the M pass's last line to reach that step and
    adds to chrom2's M copy (:1445-1451).  Returns (Imputated_Whole_Lib,
    Imputated_Local_Lib) in the reference's dense shapes."""
    from . import pairs
    genome = Load_Genome(genomeSize, chroms)
    M_M, P_P = _materialise(M_M), _materialise(P_P)
    B = pairs.PairBinner(genome, chroms)
    try:
        whole = {}
        for res in wholeRes:
            whole[res] = B.add_impute_target(res, False, UnImputated_Whole_Lib[res]["Matrix"],
                                             int(Imputation_region // res), Imputation_min, Imputation_ratio)
        local = {res: B.add_impute_target(res, True) for res in localRes}
        fm = pairs.pairs_format(pairs.ALLELIC_BED, "Both", 0, 0, mode=1, mark2="R1")
        fp = pairs.pairs_format(pairs.ALLELIC_BED, "Both", 1, 1, mode=1, mark2="R1")
        B.feed(M_M, fm)
        # the stale M_M_sub the P pass sums (NameError / IndexError where the reference has none)
        off, t = B.last_reached()
        stale = None
        if off >= 0:
            f = pairs.line_at(M_M, off).decode().strip().split()
            rl = next(r for r, tt in whole.items() if tt.index == t)
            hb, _ = pairs.haplotype_bins(genome, rl)
            s = int(Imputation_region // rl)
            c1, c2 = f[0].lstrip("chr"), f[2].lstrip("chr")
            p1, p2 = int(f[1]) // rl, int(f[3]) // rl
            U = UnImputated_Whole_Lib[rl]["Matrix"]
            if f[-1] == "R1":
                a, mb = p1 + hb["M" + c1][0], p2 + hb["M" + c2][0]
                stale = U[a - s:a + s + 1, mb - s:mb + s + 1]
            else:
                b, mb = p2 + hb["M" + c1][0], p1 + hb["M" + c2][0]
                stale = U[mb - s:mb + s + 1, b - s:b + s + 1]
        for res, tt in whole.items():
            ok, pp = False, 0
            if stale is not None:
                ii, jj = pairs.neighborhood_index(int(Imputation_region // res))
                try:
                    pp, ok = int(np.asarray(stale)[ii, jj].sum()), True
                except IndexError:
                    ok = False
            B.set_stale(tt, pp, ok)
        B.feed(P_P, fp)
        B.finish()
        IW, IL = {}, {}
        for res, tt in whole.items():
            r, c, v = B.pixels(tt)
            M = np.array(UnImputated_Whole_Lib[res]["Matrix"], dtype=np.int64, copy=True)
            np.add.at(M, (r.astype(np.int64), c.astype(np.int64)), v.astype(np.int64))
            IW[res] = {"Bins": UnImputated_Whole_Lib[res]["Bins"], "Matrix": M}
        order = B.order
        for res, tt in local.items():
            r, c, v = B.pixels(tt)
            r = r.astype(np.int64)
            IL[res] = {}
            half = int(tt.chrom_nbins.sum())
            for h, pre in enumerate("MP"):
                for k, chro in enumerate(order):
                    s0 = int(tt.chrom_first[k]) + h * half
                    n = int(tt.chrom_nbins[k])
                    lo, hi = np.searchsorted(r, [s0, s0 + n], "left")
                    M = np.array(UnImputated_Local_Lib[res][pre + chro], dtype=np.int64, copy=True)
                    np.add.at(M, (r[lo:hi] - s0, c[lo:hi].astype(np.int64) - s0), v[lo:hi].astype(np.int64))
                    IL[res][pre + chro] = M
        return IW, IL
    finally:
        B.close()


def HaplotypeMatrixBuilding(BedFiles, genomeSize, wholeRes, localRes, Imputation_region, Imputation_min,
                            Imputation_ratio, chroms):
    """The matrix part of HaplotypeMatrixBuilding (:1044-1494) on the GPU.
    BedFiles = {'Bi_Allelic', 'M_M', 'P_P', 'M_P', 'P_M': source}; returns the
    reference's DataSets dict: Tradition_Whole / _Local (all five beds,
    :1080-1095), UnImputated_Whole / _Local and Imputated_Whole / _Local."""
    from . import pairs
    srcs = {k: _materialise(v) for k, v in BedFiles.items()}
    # the traditional pass reads `cat` of the five beds in sorted file-name order (:1062, :1080-1089)
    everything = [v for k in sorted(srcs) for v in ([srcs[k]] if not isinstance(srcs[k], list) else srcs[k])]
    if all(isinstance(v, (str, os.PathLike)) for v in everything):
        trad_src = everything
    else:
        trad_src = b"".join(b"".join(pairs._iter_blocks(v, pairs.CHUNK_BYTES)) for v in everything)
    DataSets = {}
    TW, TL = TraditionalMatrixInAllelic(trad_src, genomeSize, wholeRes, localRes, chroms)
    DataSets["Tradition_Whole"], DataSets["Tradition_Local"] = TW, TL
    UW, UL = HaplotypeUnImputedBuilding(srcs["M_M"], srcs["P_P"], srcs["M_P"], srcs["P_M"], genomeSize, wholeRes,
                                        localRes, chroms)
    DataSets["UnImputated_Whole"], DataSets["UnImputated_Local"] = UW, UL
    IW, IL = HaplotypeImputation(srcs["M_M"], srcs["P_P"], genomeSize, wholeRes, localRes, chroms,
                                 Imputation_region, Imputation_min, Imputation_ratio, UW, UL)
    DataSets["Imputated_Whole"], DataSets["Imputated_Local"] = IW, IL
    return DataSets


# ------------------------------------------------- matrix construction (:617-717, :1495-1860)
# `hichap matrix` drops in here: the pairs are binned on the GPU (PairBinner),
# the tables written as multi-resolution coolers with NPZ2Cooler's layout
# (coolio / h5.py; cooler itself is absent), and `cooler balance
# --ignore-diags 1 [--cis-only] --force` replaced by coolio.balance_cooler
# (the GPU ICE path, ice.py) in place.
S_DTYPE = np.dtype({"names": ["bin1", "bin2", "IF"], "formats": [np.int64, np.int64, np.float64]})


def _chrom_ok(c, chroms):
    # NPZ2Cooler's chromosome filter (:145, :150-151, :215)
    chroms = set(chroms)
    return (not chroms) or (c.isdigit() and "#" in chroms) or (c in chroms)


def _sparse_rec(x, y, v):
    t = np.zeros(len(v), dtype=S_DTYPE)
    t["bin1"], t["bin2"], t["IF"] = x, y, v
    return t


def WholeMatrixToSparseDict(Bins, Matrix):
    """Dense whole-genome matrix -> {chrom: upper-triangle block, 'c1_c2':
    full inter block (c1 before c2 in Sort_Chromosomes order)} in
    chromosome-local bins (:457-505).  ``Matrix`` may be a torch tensor."""
    M = Matrix.cpu().numpy() if hasattr(Matrix, "cpu") else np.asarray(Matrix)
    order = Sort_Chromosomes(list(Bins))
    lib = {}
    for i, c1 in enumerate(order):
        s1, e1 = Bins[c1][0], Bins[c1][1] + 1
        for c2 in order[i:]:
            s2, e2 = Bins[c2][0], Bins[c2][1] + 1
            blk = M[s1:e1, s2:e2]
            if c1 == c2:
                blk = np.triu(blk)
            x, y = np.nonzero(blk)
            lib[c1 if c1 == c2 else c1 + "_" + c2] = _sparse_rec(x, y, blk[x, y])
    return lib


def IntraMatrixToSparseDict(Dict):
    """{chrom: dense N x N} -> {chrom: upper-triangle pixels} (:508-525)."""
    out = {}
    for chro, M in Dict.items():
        T = np.triu(M.cpu().numpy() if hasattr(M, "cpu") else np.asarray(M))
        x, y = np.nonzero(T)
        out[chro] = _sparse_rec(x, y, T[x, y])
    return out


def _genome_chromsizes(genomeSizes_file, chroms):
    """NPZ2Cooler.readChromSize (:212-223), Sort_Chromosomes order (:135-138)."""
    lines = open(genomeSizes_file) if isinstance(genomeSizes_file, (str, os.PathLike)) else genomeSizes_file
    sizes = {}
    try:
        for line in lines:
            if isinstance(line, bytes):
                line = line.decode()
            f = line.strip().split()
            if f and _chrom_ok(f[0].lstrip("chr"), chroms):
                sizes[f[0].lstrip("chr")] = int(f[1])
    finally:
        if isinstance(genomeSizes_file, (str, os.PathLike)):
            lines.close()
    return [(c, sizes[c]) for c in Sort_Chromosomes(list(sizes))]


def _upper_sum(x, y, v, n):
    """Sum equal (x, y) pixels; (key-sorted) arrays."""
    if x.size == 0:
        return x, y, v
    key = x * n + y
    uk, inv = np.unique(key, return_inverse=True)
    return uk // n, uk % n, np.bincount(inv, v, minlength=uk.size)


def npz2cooler_tables(datasets, genomeSizes_file, chroms=("#", "X"), onlyIntra=True, dtype="int"):
    """The pixel tables NPZ2Cooler writes (:100-303), one per resolution:
    {res: (chromsizes [(name, length)], bin1, bin2, count)}.  Bins are
    cooler's ``binnify`` (ceil(length / res) per chromosome, only the
    chromosomes the data names); each block's local bins are offset by the
    cumulative bin counts exactly as ``_generator`` offsets them (:296-299),
    the intra blocks symmetrised then cut to the upper triangle (a lower
    entry's value lands on its mirror, :290-293), pixels sorted by (bin1,
    bin2) with equal ones summed (create_from_unordered's merge).  count is
    int32 for dtype 'int' (traditional / unimputed), float64 otherwise."""
    full = _genome_chromsizes(genomeSizes_file, chroms)
    names = [c for c, _ in full]
    out = {}
    for res, lib in datasets.items():
        Map = {}
        for key in lib:
            if "_" not in key and _chrom_ok(key, chroms):
                Map[(key, key)] = key
                continue
            part = key.split("_")
            if len(part) == 2 and _chrom_ok(part[0], chroms) and _chrom_ok(part[1], chroms):
                Map[(part[0], part[1])] = key
        subset = {c for pair in Map for c in pair}
        cs = [(c, L) for c, L in full if c in subset]
        cum = np.cumsum([-(-L // res) for _, L in cs]).astype(np.int64)  # bin_cumnums (:225-235)
        nb = int(cum[-1]) if cum.size else 0
        xs, ys, vs = [], [], []
        for i, ci_name in enumerate(names):
            for j in range(i, len(names)):
                c1, c2 = ci_name, names[j]
                if onlyIntra and c1 != c2:
                    continue
                ci, cj = i, j
                if (c1, c2) not in Map:
                    if (c2, c1) not in Map:
                        continue
                    c1, c2, ci, cj = c2, c1, j, i
                d = lib[Map[(c1, c2)]]
                x = np.asarray(d["bin1"], np.int64)
                y = np.asarray(d["bin2"], np.int64)
                v = np.asarray(d["IF"], np.float64)
                if x.size == 0:
                    continue
                if ci > cj:
                    x, y, ci, cj = y, x, cj, ci
                if ci == cj:
                    # lil: M[y, x] = M[x, y] then triu (:290-293): the upper
                    # cell takes its lower mirror's value where one exists
                    L = int(max(x.max(), y.max())) + 1
                    x, y, v = _upper_sum(x, y, v, L)
                    low = x > y
                    ux, uy = np.where(low, y, x), np.where(low, x, y)
                    o = np.lexsort((~low, uy, ux))  # per cell: the lower entry first
                    ux, uy, v = ux[o], uy[o], v[o]
                    first = np.ones(ux.size, bool)
                    first[1:] = (ux[1:] != ux[:-1]) | (uy[1:] != uy[:-1])
                    x, y, v = ux[first], uy[first], v[first]
                else:
                    x, y, v = _upper_sum(x, y, v, int(y.max()) + 1)
                nz = v != 0
                x, y, v = x[nz], y[nz], v[nz]
                if ci > 0:
                    x = x + cum[ci - 1]  # (positional, as the reference's Series access)
                if cj > 0:
                    y = y + cum[cj - 1]
                xs.append(x)
                ys.append(y)
                vs.append(v)
        if xs:
            b1, b2, val = _upper_sum(np.concatenate(xs), np.concatenate(ys), np.concatenate(vs),
                                     max(nb, int(max(map(np.max, ys)))) + 1)
        else:
            b1 = b2 = np.zeros(0, np.int64)
            val = np.zeros(0)
        out[res] = (cs, b1, b2, val.astype(np.int32) if dtype == "int" else val.astype(np.float64))
    return out


class NPZ2Cooler:
    """Save the reference's sparse dicts into a multi-resolution cooler
    (:100-210): ``datasets`` = {res: lib}, one ``outfil::res`` group per
    resolution, appended to an existing file (mode 'a'); metadata
    {'onlyIntra': str(onlyIntra)} as the reference stores it."""

    def __init__(self, datasets, outfil, genomeSizes_file, chroms=("#", "X"), onlyIntra=True, dtype="int"):
        from . import coolio
        self.outfil = os.path.abspath(os.path.expanduser(outfil))
        self.onlyIntra = onlyIntra
        tabs = npz2cooler_tables(datasets, genomeSizes_file, chroms, onlyIntra, dtype)
        meta = {"onlyIntra": str(onlyIntra)}
        coolio.create_cooler(self.outfil, {res: t + (meta,) for res, t in tabs.items()}, mode="a")


def _write_coolers(outfil, parts, genomeSize, chroms):
    """Several NPZ2Cooler calls into one file as ONE write (every
    append rewrites the whole file, so one call per part made the file I/O
    quadratic in the resolutions): ``parts`` = [(datasets, onlyIntra, dtype)],
    the same groups, tables and metadata as the calls one after the other."""
    from . import coolio
    spec = {}
    for datasets, onlyIntra, dtype in parts:
        meta = {"onlyIntra": str(onlyIntra)}
        for res, t in npz2cooler_tables(datasets, genomeSize, chroms, onlyIntra, dtype).items():
            spec[res] = t + (meta,)
    coolio.create_cooler(os.path.abspath(os.path.expanduser(outfil)), spec, mode="a")


def merge_coolers(output_uri, input_uris, write=True):
    """cooler.merge_coolers as TraditionalMatrixConstruction calls it
    (:680-695): the inputs' pixels of one resolution summed into
    ``output_uri`` (appended to its file); every input must have the same
    bins.  write=False: return (group, table spec) instead, for one
    create_cooler over every resolution."""
    from . import coolio
    tabs, cs, meta = [], None, None
    for uri in input_uris:
        with coolio.Cooler(uri) as c:
            cur = [(n, int(c.chromsizes[n])) for n in c.chromnames]
            if cs is not None and (cur != cs or c.binsize != binsize):
                raise ValueError(f"merge_coolers: {uri} has different bins")
            cs, binsize = cur, c.binsize
            meta = c.info.get("metadata")
            tabs.append(c.pixels_table())
    b1 = np.concatenate([np.asarray(t[0], np.int64) for t in tabs])
    b2 = np.concatenate([np.asarray(t[1], np.int64) for t in tabs])
    dt = tabs[0][2].dtype
    v = np.concatenate([np.asarray(t[2], np.float64) for t in tabs])
    n = int(sum(-(-L // binsize) for _, L in cs)) + 1
    b1, b2, v = _upper_sum(b1, b2, v, max(n, int(b2.max(initial=0)) + 1))
    path, grp = output_uri.split("::") if "::" in output_uri else (output_uri, str(binsize))
    try:
        meta = json.loads(meta) if isinstance(meta, str) else meta
    except ValueError:
        meta = None
    if not write:
        return path, grp, (cs, b1, b2, v.astype(dt), meta)
    coolio.create_cooler(path, {grp: (cs, b1, b2, v.astype(dt), meta)}, mode="a")


def _merge_all(merged, reps, resolutions):
    """merge_coolers for every resolution into ``merged`` as one write."""
    from . import coolio
    spec = {}
    for res in resolutions:
        _, grp, t = merge_coolers(f"{merged}::{res}", [f"{r}::{res}" for r in reps], write=False)
        spec[grp] = t
    coolio.create_cooler(merged, spec, mode="a")


def _balance_all(coolers, wholeRes, localRes):
    """The `cooler balance --ignore-diags 1 [--cis-only] --force` calls
    (:699-714, :1533-1544): genome-wide for wholeRes, --cis-only for
    localRes, weights written in place."""
    from . import coolio
    for res in wholeRes:
        for f in coolers:
            coolio.balance_cooler(f"{f}::{res}", ignore_diags=1, cis_only=False)
    for res in localRes:
        for f in coolers:
            coolio.balance_cooler(f"{f}::{res}", ignore_diags=1, cis_only=True)


def TraditionalMatrixConstruction(OutPath, RepPath, genomeSize, wholeRes, localRes, chroms=("#", "X"),
                                  balance=True):
    """`hichap matrix` for traditional (non-allelic) data (:617-717): per
    replicate directory every ``*_Valid.bed`` binned on the GPU (all files
    of a replicate together, as the reference's ``cat``), written to
    ``OutPath/Cooler/<prefix>Multi.cool`` (whole-genome groups for wholeRes,
    intra-chromosome groups for localRes), the replicates merged into
    ``Merged_Multi.cool``, then every cooler balanced in place.  Returns the
    cooler paths (replicates, then merged).  (The reference takes the bed
    files in os.listdir order; sorted here -- the counts do not depend on it,
    the prefix is the first name.)"""
    CoolerPath = os.path.join(OutPath, "Cooler")
    os.makedirs(CoolerPath, exist_ok=True)
    reps = []
    for rep_p in RepPath:
        files = sorted(i for i in os.listdir(rep_p) if "_Valid.bed" in i)
        if not files:
            raise FileNotFoundError(f"no *_Valid.bed in {rep_p}")
        prefix = files[0].split("Valid")[0]
        Whole_Lib, Local_Lib = TraditionalMatrixBuilding([os.path.join(rep_p, f) for f in files], genomeSize,
                                                         wholeRes, localRes, chroms)
        out = os.path.join(CoolerPath, prefix + "Multi.cool")
        if os.path.exists(out):
            os.remove(out)  # written afresh (the reference appends into an existing file)
        _write_coolers(out, [(Whole_Lib, False, "int"), (Local_Lib, True, "int")], genomeSize, chroms)
        reps.append(out)
    merged = os.path.join(CoolerPath, "Merged_Multi.cool")
    if os.path.exists(merged):
        os.remove(merged)
    _merge_all(merged, reps, list(wholeRes) + list(localRes))
    coolers = reps + [merged]
    if balance:
        _balance_all(coolers, wholeRes, localRes)
    return coolers


def _hap_genome(genomeSize, chroms, out_path):
    """Hap_genomeSize (:1551-1565): 'M' + chrom and 'P' + chrom lines."""
    lines = open(genomeSize).read().splitlines() if isinstance(genomeSize, (str, os.PathLike)) else \
        [x.decode() if isinstance(x, bytes) else x for x in genomeSize]
    hap, names = [], []
    for line in lines:
        f = line.strip().split()
        if not f:
            continue
        f[0] = f[0].lstrip("chr")
        if _chrom_ok(f[0], chroms):
            names += ["M" + f[0], "P" + f[0]]
            hap += ["M" + "\t".join(f) + "\n", "P" + "\t".join(f) + "\n"]
    with open(out_path, "w") as fh:
        fh.writelines(hap)
    return out_path, names


def _haplotype_coolers(OutPath, prefix, genomeSize, wholeRes, localRes, chroms, DataSets):
    """The cooler part of HaplotypeMatrixBuilding (:1501-1638) on its
    DataSets: traditional cooler (int, ICE-balanced in place), unimputed
    haplotype cooler (int), two-step corrected imputed haplotype cooler
    (float: GenomeWideMatrixCorrection per wholeRes, IntraChromMatrixCorrection
    per localRes) and the gap file ``<prefix>Imputated_Gap.npz``."""
    trad = os.path.join(OutPath, prefix + "Traditional_Multi.cool")
    for f in (trad,):
        if os.path.exists(f):
            os.remove(f)
    W = {res: WholeMatrixToSparseDict(DataSets["Tradition_Whole"][res]["Bins"],
                                      DataSets["Tradition_Whole"][res]["Matrix"]) for res in wholeRes}
    L = {res: IntraMatrixToSparseDict(DataSets["Tradition_Local"][res]) for res in localRes}
    _write_coolers(trad, [(W, False, "int"), (L, True, "int")], genomeSize, chroms)
    _balance_all([trad], wholeRes, localRes)
    hap_gs, hap_chroms = _hap_genome(genomeSize, chroms, os.path.join(OutPath, "Hap_genomeSize"))
    unimp = os.path.join(OutPath, prefix + "UnImputated_Haplotype_Multi.cool")
    imp = os.path.join(OutPath, prefix + "Imputated_Haplotype_Multi.cool")
    for f in (unimp, imp):
        if os.path.exists(f):
            os.remove(f)
    W = {res: WholeMatrixToSparseDict(DataSets["UnImputated_Whole"][res]["Bins"],
                                      DataSets["UnImputated_Whole"][res]["Matrix"]) for res in wholeRes}
    L = {res: IntraMatrixToSparseDict(DataSets["UnImputated_Local"][res]) for res in localRes}
    _write_coolers(unimp, [(W, False, "int"), (L, True, "int")], hap_gs, hap_chroms)
    BW = {}
    for res in wholeRes:
        hb = DataSets["Imputated_Whole"][res]["Bins"]
        Bal = GenomeWideMatrixCorrection(DataSets["Tradition_Whole"][res]["Bins"], hb,
                                         DataSets["Tradition_Whole"][res]["Matrix"],
                                         DataSets["Imputated_Whole"][res]["Matrix"])
        BW[res] = WholeMatrixToSparseDict(hb, Bal)
    BL, Gap_Local = {}, {}
    for res in localRes:
        Nor_Lib, Gap_Lib = IntraChromMatrixCorrection(DataSets["Tradition_Local"][res],
                                                      DataSets["Imputated_Local"][res])
        BL[res] = IntraMatrixToSparseDict(Nor_Lib)
        Gap_Local[str(res)] = Gap_Lib
    # np.savez of the per-resolution dicts, as the reference saves them (:1616-1617)
    np.savez(os.path.join(OutPath, prefix + "Imputated_Gap.npz"),
             **{k: np.array(v, dtype=object) for k, v in Gap_Local.items()})
    _write_coolers(imp, [(BW, False, "float"), (BL, True, "float")], hap_gs, hap_chroms)
    return trad, unimp, imp


_HAP_BEDS = ("Bi_Allelic", "M_M", "M_P", "P_P", "P_M")


def _haplotype_bed_files(BedPath):
    """The five allelic beds of a replicate directory (:1061-1074)."""
    files = sorted(i for i in os.listdir(BedPath) if any(k + ".bed" in i for k in _HAP_BEDS))
    found = {k: [os.path.join(BedPath, f) for f in files if k + ".bed" in f] for k in _HAP_BEDS}
    for k in ("Bi_Allelic", "M_M", "M_P", "P_P", "P_M"):
        if not found[k]:
            raise FileNotFoundError(f"Missing file {k}.bed in {BedPath}")
    return files[0].split("Valid")[0], {k: v if len(v) > 1 else v[0] for k, v in found.items()}


def HaplotypeMatrixConstruction(OutPath, RepPath, genomeSize, wholeRes, localRes, Imputation_region=10000000,
                                Imputation_min=2, Imputation_ratio=0.9, chroms=("#", "X")):
    """`hichap matrix` for haplotype-resolved data (:1641-1860): per replicate
    the GPU builds the traditional, unimputed and imputed matrices
    (HaplotypeMatrixBuilding), writes its three coolers + gap file under
    ``OutPath/Cooler`` (traditional ICE-balanced in place, imputed two-step
    corrected); with several replicates their matrices are summed and the
    same is written with prefix ``Merged_``.  Returns {prefix: (traditional,
    unimputed, imputed) cooler paths}.  (The reference's one-replicate path
    omits genomeSize and raises TypeError, :1676-1683; here it runs.)"""
    CoolerPath = os.path.join(OutPath, "Cooler")
    os.makedirs(CoolerPath, exist_ok=True)
    out, All = {}, None
    for rep_p in RepPath:
        prefix, beds = _haplotype_bed_files(rep_p)
        DataSets = HaplotypeMatrixBuilding(beds, genomeSize, wholeRes, localRes, Imputation_region, Imputation_min,
                                           Imputation_ratio, chroms)
        out[prefix] = _haplotype_coolers(CoolerPath, prefix, genomeSize, wholeRes, localRes, chroms, DataSets)
        if len(RepPath) == 1:
            return out
        if All is None:
            All = DataSets
        else:
            for kind in ("Tradition", "UnImputated", "Imputated"):
                for res in wholeRes:
                    All[kind + "_Whole"][res]["Matrix"] = All[kind + "_Whole"][res]["Matrix"] + \
                        DataSets[kind + "_Whole"][res]["Matrix"]
                for res in localRes:
                    for k in All[kind + "_Local"][res]:
                        All[kind + "_Local"][res][k] = All[kind + "_Local"][res][k] + DataSets[kind + "_Local"][res][k]
    out["Merged_"] = _haplotype_coolers(CoolerPath, "Merged_", genomeSize, wholeRes, localRes, chroms, All)
    return out
