"""ICE balancing on MI355X — drop-in for HiCHap's ``cooler balance`` calls.

HiCHap balances every traditional cooler with the third-party CLI

    cooler balance --ignore-diags 1 --force          <file>::<wholeRes>
    cooler balance --ignore-diags 1 --cis-only --force <file>::<localRes>

(matrixBuilding.py:708, :713, :1537, :1542, :1761, :1766).  ``balance`` below
takes the same pixel table cooler reads (``pixels/bin1_id``, ``bin2_id``,
``count``) plus ``indexes/chrom_offset`` and returns what cooler writes to
``bins/weight`` and its attrs.  The whole iteration runs in HBM on the
pixel-chunk layout; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import asdict, dataclass

import numpy as np

from . import _lib
from ._lib import IceOpts, MatrixInfo, SynthParams, call, ptr


@dataclass
class IceOptions:
    """cooler ``balance_cooler`` keyword defaults with HiCHap's overrides
    (``ignore_diags=1``; ``cis_only`` for the local resolutions)."""
    ignore_diags: int = 1
    cis_only: bool = False
    mad_max: int = 5
    min_nnz: int = 10
    min_count: float = 0
    tol: float = 1e-5
    max_iters: int = 200
    rescale_marginals: bool = True
    check_every: int = 8

    def c_opts(self) -> IceOpts:
        return IceOpts(int(self.mad_max), int(self.min_nnz), float(self.min_count), float(self.tol),
                       int(self.max_iters), int(bool(self.rescale_marginals)),
                       int(self.check_every), 0)


class ContactMatrix:
    """A contact matrix resident in HBM in the pixel-chunk layout (owns an
    ``hh_matrix*``).  Rows ``[row_lo, row_hi)`` are held (a shard for
    multi-GPU genome-wide ICE)."""

    def __init__(self, handle, chrom_offsets):
        self._h = handle
        self.chrom_offsets = np.asarray(chrom_offsets, dtype=np.int64)

    # ---------------------------------------------------------------- build
    @classmethod
    def from_pixels(cls, bin1, bin2, count, n_bins, chrom_offsets, ignore_diags=1,
                    cis_only=False, row_range=None, stream=None):
        _lib.require_gpu()
        b1 = np.ascontiguousarray(bin1, dtype=np.int64)
        b2 = np.ascontiguousarray(bin2, dtype=np.int64)
        cnt = np.ascontiguousarray(count, dtype=np.float64)
        if not (b1.shape == b2.shape == cnt.shape):
            raise ValueError("bin1, bin2 and count must have the same length")
        off = np.ascontiguousarray(chrom_offsets, dtype=np.int64)
        lo, hi = (0, int(n_bins)) if row_range is None else (int(row_range[0]), int(row_range[1]))
        h = C.c_void_p()
        call("hh_matrix_from_pixels", ptr(b1), ptr(b2), ptr(cnt), b1.size, int(n_bins), ptr(off),
             off.size - 1, int(ignore_diags), int(bool(cis_only)), lo, hi, stream, C.byref(h))
        return cls(h, off)

    @classmethod
    def from_device_pixels(cls, bin1, bin2, count, n_bins, chrom_offsets, ignore_diags=1, cis_only=False,
                           row_range=None, stream=None, nnz=None):
        """Build from a pixel table already in HBM (cooler order: sorted by
        (bin1, bin2), bin1 <= bin2, unique; int32 ids and counts) — e.g. the
        output of ``PairBinner`` — with no host round trip.  ``bin1`` /
        ``bin2`` / ``count`` are int32 torch tensors or raw device pointers
        (then ``nnz`` is required)."""
        _lib.require_gpu()
        def dptr(x):
            if hasattr(x, "data_ptr"):
                import torch
                if x.dtype != torch.int32 or not x.is_cuda or not x.is_contiguous():
                    raise ValueError("expected contiguous int32 device tensors")
                return C.c_void_p(x.data_ptr()), int(x.numel())
            return C.c_void_p(int(x)), None
        (p1, n1), (p2, n2), (pc, n3) = dptr(bin1), dptr(bin2), dptr(count)
        n = nnz if nnz is not None else n1
        if n is None or (n1 is not None and not (n1 == n2 == n3 == n)):
            raise ValueError("bin1, bin2 and count must have the same length (nnz)")
        off = np.ascontiguousarray(chrom_offsets, dtype=np.int64)
        lo, hi = (0, int(n_bins)) if row_range is None else (int(row_range[0]), int(row_range[1]))
        h = C.c_void_p()
        call("hh_matrix_from_pixels_device", p1, p2, pc, int(n), int(n_bins), ptr(off), off.size - 1,
             int(ignore_diags), int(bool(cis_only)), lo, hi, stream, C.byref(h))
        return cls(h, off)

    @classmethod
    def synthetic(cls, chrom_nbins, row_range=None, stream=None, **kw):
        """Generate a synthetic genome in HBM (see synth_params); rows
        ``row_range`` (aligned to 512-row blocks) or all."""
        _lib.require_gpu()
        p, keep = synth_params(chrom_nbins, **kw)
        n = int(np.sum(chrom_nbins))
        lo, hi = (0, n) if row_range is None else (int(row_range[0]), int(row_range[1]))
        h = C.c_void_p()
        call("hh_synth_build", C.byref(p), lo, hi, stream, C.byref(h))
        off = np.concatenate([[0], np.cumsum(chrom_nbins)]).astype(np.int64)
        return cls(h, off)

    # ----------------------------------------------------------------- info
    @property
    def handle(self):
        return self._h

    def info(self) -> dict:
        inf = MatrixInfo()
        call("hh_matrix_get_info", self._h, C.byref(inf))
        return {k: getattr(inf, k) for k, _ in MatrixInfo._fields_}

    def export_upper(self):
        """Stored upper-triangle pixels back on the host (checking only)."""
        n = C.c_int64(0)
        call("hh_matrix_export_upper", self._h, None, None, None, C.byref(n))
        b1 = np.empty(n.value, np.int64)
        b2 = np.empty(n.value, np.int64)
        c = np.empty(n.value, np.float64)
        call("hh_matrix_export_upper", self._h, ptr(b1), ptr(b2), ptr(c), C.byref(n))
        return b1, b2, c

    def close(self):
        if self._h:
            call("hh_matrix_free", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def synth_params(chrom_nbins, A=30.0, decay=1.08, comp_strength=0.3, vis_sigma=0.3, gap_frac=0.02,
                 trans_density=0.0, comp_block=200, ignore_diags=1, cis_only=False, seed=20201015):
    arr = np.ascontiguousarray(chrom_nbins, dtype=np.int32)
    p = SynthParams(arr.size, arr.ctypes.data_as(C.POINTER(C.c_int32)), float(A), float(decay),
                    float(comp_strength), float(vis_sigma), float(gap_frac), float(trans_density),
                    int(comp_block), int(ignore_diags), int(bool(cis_only)), 0, int(seed))
    return p, arr  # keep `arr` alive while p is used


class DevArray:
    """A device buffer view (pointer, length, dtype) with the torch-like
    ``data_ptr()`` / ``numel()`` the table-driven entry points accept."""

    def __init__(self, p, n, owner=None):
        self._p, self._n, self._owner = int(p or 0), int(n), owner

    def data_ptr(self):
        return self._p

    def numel(self):
        return self._n


class SynthPixels:
    """Synthetic pixel table in HBM (hh_synth_pixels): cooler's upper-triangle
    table, or with ``ordered`` every cell of an asymmetric matrix."""

    def __init__(self, chrom_nbins, ordered=False, stream=None, **kw):
        _lib.require_gpu()
        p, keep = synth_params(chrom_nbins, **kw)
        h = C.c_void_p()
        call("hh_synth_pixels", C.byref(p), int(bool(ordered)), stream, C.byref(h))
        self._h = h
        p1, p2, pc, n = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_int64(0)
        call("hh_pixels_get", h, C.byref(p1), C.byref(p2), C.byref(pc), C.byref(n))
        self.nnz = int(n.value)
        self.bin1, self.bin2, self.count = (DevArray(x.value, self.nnz, self) for x in (p1, p2, pc))

    def close(self):
        if self._h:
            call("hh_pixels_free", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def synth_dense(chrom_nbins, chrom, out_ptr, stream=None, **kw):
    """Dense float64 cis block of chromosome ``chrom`` of the synthetic genome
    written to device memory at ``out_ptr`` (N_c x N_c, row-major)."""
    _lib.require_gpu()
    p, keep = synth_params(chrom_nbins, **kw)
    call("hh_synth_dense", C.byref(p), int(chrom), C.c_void_p(int(out_ptr)), stream)


def synth_row_counts(chrom_nbins, stream=None, **kw):
    """Counting pass of the generator: per-row stored slots (work) and
    upper-triangle pixel counts for every row (used to partition rows)."""
    _lib.require_gpu()
    p, keep = synth_params(chrom_nbins, **kw)
    n = int(np.sum(chrom_nbins))
    rc = np.empty(n, np.int32)
    ru = np.empty(n, np.int64)
    call("hh_synth_count", C.byref(p), ptr(rc), ptr(ru), stream)
    return rc, ru


def _stats(opts: IceOptions, scale, var, iters, conv, cis_only):
    st = dict(tol=opts.tol, min_nnz=opts.min_nnz, min_count=opts.min_count, mad_max=opts.mad_max,
              cis_only=bool(cis_only), ignore_diags=opts.ignore_diags, divisive_weights=False)
    if cis_only:
        st.update(scale=scale.copy(), var=float(var[-1]) if len(var) else float("nan"),
                  converged=bool(var[-1] < opts.tol) if len(var) else False,
                  iters=iters.copy(), chrom_converged=conv.astype(bool), chrom_var=var.copy())
    else:
        st.update(scale=float(scale[0]), var=float(var[0]), converged=bool(conv[0]), iters=int(iters[0]))
    return st


def balance_matrix(m: ContactMatrix, opts: IceOptions | None = None, stream=None):
    """Balance a matrix that holds every row, on one GPU.
    Returns ``(weights, stats)`` like cooler's ``balance_cooler``."""
    opts = opts or IceOptions()
    inf = m.info()
    G = inf["n_chroms"] if inf["cis_only"] else 1
    w = np.empty(inf["n_bins"], np.float64)
    scale, var = np.empty(G), np.empty(G)
    iters, conv = np.empty(G, np.int32), np.empty(G, np.int32)
    secs = C.c_double(0)
    call("hh_ice_balance", m.handle, C.byref(opts.c_opts()), ptr(w), ptr(scale), ptr(var), ptr(iters),
         ptr(conv), C.byref(secs), stream)
    st = _stats(opts, scale, var, iters, conv, inf["cis_only"])
    st["sweep_seconds"] = secs.value
    return w, st


def balance(bin1, bin2, count, n_bins, chrom_offsets, ignore_diags=1, cis_only=False, mad_max=5,
            min_nnz=10, min_count=0, tol=1e-5, max_iters=200, rescale_marginals=True, stream=None):
    """cooler ``balance_cooler`` on the GPU from the pixel table.

    Equivalent of ``cooler balance --ignore-diags {ignore_diags} [--cis-only]``
    as HiCHap invokes it (matrixBuilding.py:706-714). Returns (weights, stats).
    """
    opts = IceOptions(ignore_diags=ignore_diags, cis_only=cis_only, mad_max=mad_max, min_nnz=min_nnz,
                      min_count=min_count, tol=tol, max_iters=max_iters,
                      rescale_marginals=rescale_marginals)
    m = ContactMatrix.from_pixels(bin1, bin2, count, n_bins, chrom_offsets, ignore_diags, cis_only,
                                  stream=stream)
    try:
        return balance_matrix(m, opts, stream)
    finally:
        m.close()


def cooler_balance_cmd(pixels, chrom_offsets, n_bins, ignore_diags=1, cis_only=False, **kw):
    """The HiCHap call-site form: ``pixels`` is a mapping with cooler's column
    names (``bin1_id``, ``bin2_id``, ``count``); returns (weights, stats)."""
    return balance(pixels["bin1_id"], pixels["bin2_id"], pixels["count"], n_bins, chrom_offsets,
                   ignore_diags=ignore_diags, cis_only=cis_only, **kw)


class IceState:
    """Device ICE state for the sharded (multi-GPU) driver; wraps ``hh_ice*``."""

    def __init__(self, m: ContactMatrix, opts: IceOptions):
        self.m = m
        self.opts = opts
        h = C.c_void_p()
        call("hh_ice_create", m.handle, C.byref(opts.c_opts()), C.byref(h))
        self._h = h
        g = C.c_int32(0)
        call("hh_ice_n_groups", h, C.byref(g))
        self.n_groups = g.value

    def marg_local(self, mode, out=None, stream=None):
        call("hh_ice_marg_local", self._h, int(mode), ptr(out), stream)

    def bind_exchange(self, ex):
        """Register ``ex``'s int64 reduce-scatter for the column side of the
        upper-triangle tiles (hh_ice_set_column_exchange; a no-op for a
        whole matrix or a layout without them)."""
        if ex.world <= 1:
            return
        self._rs = ex.reduce_callback()  # kept alive with the state
        rr = np.ascontiguousarray(ex.rank_rows, dtype=np.int64)
        call("hh_ice_set_column_exchange", self._h, int(ex.world), -1, ptr(rr), C.cast(self._rs, C.c_void_p),
             None, None, None)

    def set_marg(self, gathered, world, maxlen, rank_rows, stream=None):
        rr = np.ascontiguousarray(rank_rows, dtype=np.int64)
        call("hh_ice_set_marg", self._h, ptr(gathered), int(world), int(maxlen), ptr(rr), stream)

    def filter_nnz(self, stream=None):
        call("hh_ice_filter_nnz", self._h, stream)

    def filter_count_mad(self, stream=None):
        call("hh_ice_filter_count_mad", self._h, stream)

    def update(self, stream=None):
        call("hh_ice_update", self._h, stream)

    def active_groups(self, stream=None) -> int:
        n = C.c_int32(0)
        call("hh_ice_active_groups", self._h, C.byref(n), stream)
        return n.value

    def iterations_done(self) -> int:
        n = C.c_int32(0)
        call("hh_ice_iterations_done", self._h, C.byref(n))
        return n.value

    def run(self, n, stream=None):
        call("hh_ice_run", self._h, int(n), stream)

    def last_timing(self):
        ms, k, it = C.c_double(0), C.c_int32(0), C.c_double(0)
        call("hh_ice_last_sweep_timing", self._h, C.byref(ms), C.byref(k), C.byref(it))
        return ms.value, k.value, it.value

    def swept_bytes(self):
        """Payload bytes one sweep reads (hh_ice_swept_bytes)."""
        b = C.c_int64(0)
        call("hh_ice_swept_bytes", self._h, C.byref(b))
        return b.value

    def bias(self, stream=None):
        """The current bias vector b (n_bins, host; checking only)."""
        b = np.empty(int(self.m.info()["n_bins"]))
        call("hh_ice_get_bias", self._h, ptr(b), stream)
        return b

    def finalize(self, stream=None):
        n = int(self.m.info()["n_bins"])
        G = self.n_groups
        w = np.empty(n)
        scale, var = np.empty(G), np.empty(G)
        iters, conv = np.empty(G, np.int32), np.empty(G, np.int32)
        call("hh_ice_finalize", self._h, ptr(w), ptr(scale), ptr(var), ptr(iters), ptr(conv), stream)
        return w, _stats(self.opts, scale, var, iters, conv, self.m.info()["cis_only"])

    def close(self):
        if self._h:
            call("hh_ice_free", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


__all__ = ["IceOptions", "ContactMatrix", "IceState", "SynthPixels", "DevArray", "balance", "balance_matrix",
           "cooler_balance_cmd", "synth_row_counts", "synth_params", "asdict"]
