"""Pair binning on the GPU: HiCHap pair text -> contact matrices (cooler
pixel tables), through the ``hh_binner_*`` C-ABI (csrc/pairs.hip).

Reference loops replaced (HiCHap/matrixBuilding.py):

* ``TraditionalMatrixBuilding``   :528-596 (fields 1, 6, 8, 13 of *_Valid.bed)
* ``TraditionalMatrixInAllelic``  :793-854 (fields 0-3 of the allelic beds)
* ``HaplotypeMatrixBuilding``     :1126-1240 (unimputed M_M / P_P passes keep
  only lines whose last field is ``Both``; M_P / P_M bin chrom1 and chrom2 in
  different haplotype halves and build no intra-chromosome matrix)

The reference fills dense N x N int matrices one line at a time; here every
line becomes the key of its unordered bin pair, the keys are radix-sorted and
run-length encoded on the GPU, and the result is the upper-triangle pixel
table (bin1 <= bin2, counts).  The same-named functions in
``hichap_master_amd.matrixBuilding`` turn pixel tables into the reference's
return shapes.  There is no CPU fallback: without the library or a GPU every
call raises.
"""
from __future__ import annotations

import ctypes as C
import io
import os
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import call, ptr

CHUNK_BYTES = 256 << 20


class PairsFormat(C.Structure):
    _fields_ = [("col_chrom1", C.c_int32), ("col_pos1", C.c_int32), ("col_chrom2", C.c_int32),
                ("col_pos2", C.c_int32), ("mark", C.c_char * 16), ("hap1", C.c_int32), ("hap2", C.c_int32),
                ("mode", C.c_int32), ("mark2", C.c_char * 16)]


# field layouts of the reference's pair files
VALID_BED = (1, 6, 8, 13)     # TraditionalMatrixBuilding :577-588
ALLELIC_BED = (0, 1, 2, 3)    # TraditionalMatrixInAllelic :824-836, haplotype passes :1135-1142


def pairs_format(cols=VALID_BED, mark="", hap1=0, hap2=0, mode=0, mark2="") -> PairsFormat:
    m, m2 = mark.encode(), mark2.encode()
    if len(m) > 15 or len(m2) > 15:
        raise ValueError("mark longer than 15 bytes")
    return PairsFormat(cols[0], cols[1], cols[2], cols[3], m, int(hap1), int(hap2), int(mode), m2)


# ----------------------------------------------------------- genome / bins
def strip_chr(name: str) -> str:
    """``str.lstrip('chr')``: removes any leading 'c', 'h', 'r' characters."""
    return name.lstrip("chr")


def _passes(c: str, chroms) -> bool:
    """The reference's chromosome filter (:357-358, :577-580)."""
    return (not chroms) or (c.isdigit() and ("#" in chroms)) or (c in chroms)


def load_genome(genomeSize, chroms) -> dict:
    """Load_Genome (:349-366): {stripped name: length} for accepted chroms.
    ``genomeSize`` is a path or an iterable of lines."""
    genome = {}
    lines = open(genomeSize, "r") if isinstance(genomeSize, (str, os.PathLike)) else genomeSize
    try:
        for line in lines:
            if isinstance(line, bytes):
                line = line.decode()
            f = line.strip().split()
            c = f[0].lstrip("chr")
            if _passes(c, chroms):
                genome[c] = int(f[1])
    finally:
        if isinstance(genomeSize, (str, os.PathLike)):
            lines.close()
    return genome


def sort_chromosomes(names):
    """Sort_Chromosomes (:388-406): numeric labels ascending, then the rest."""
    names = [i.lstrip("chr") for i in names]
    num, st = [], []
    for i in names:
        try:
            num.append(int(i))
        except ValueError:
            st.append(i)
    num.sort()
    st.sort()
    return [str(j) for j in num] + st


def chrom_bins(genome: dict, res: int):
    """Get_Chro_Bins (:409-426): ({chrom: (first, last)} inclusive, total)."""
    order = sort_chromosomes(genome)
    bins, s = {}, 0
    for c in order:
        n = genome[c] // res + 1
        bins[c] = (s, s + n - 1)
        s += n
    return bins, s


def haplotype_bins(genome: dict, res: int):
    """Get_Chro_Bins_Haplotypes (:429-454): 'M'+c for every chrom, then 'P'+c."""
    order = sort_chromosomes(genome)
    bins, s = {}, 0
    for h in ("M", "P"):
        for c in order:
            n = genome[c] // res + 1
            bins[h + c] = (s, s + n - 1)
            s += n
    return bins, s


@dataclass
class Target:
    """One output matrix: resolution, whole-genome or intra-chromosome,
    traditional (n bins) or haplotype (M half then P half) layout."""
    res: int
    local: bool
    haplotype: bool
    index: int = -1


def _name_table(genome: dict, chroms):
    order = sort_chromosomes(genome)
    ids = {c: k for k, c in enumerate(order)}
    names = list(order)
    codes = [ids[c] for c in order]
    # names the filter accepts but genomeSize lacks: the reference raises KeyError
    for c in (chroms or []):
        if c != "#" and c not in ids:
            names.append(c)
            codes.append(-2)
    if not chroms:
        policy = 2
    elif "#" in chroms:
        policy = 1
    else:
        policy = 0
    return order, names, codes, policy


def _iter_blocks(source, chunk):
    """Yield byte blocks of a pair source with `cat` semantics: a path, a list
    of paths, bytes-like, a binary/text file object, or an iterable of lines."""
    if isinstance(source, (bytes, bytearray, memoryview)):
        yield bytes(source)
        return
    if isinstance(source, (str, os.PathLike)):
        with open(source, "rb") as f:
            while True:
                b = f.read(chunk)
                if not b:
                    return
                yield b
        return
    if (isinstance(source, (list, tuple)) and source
            and all(isinstance(s, (str, os.PathLike)) and os.path.isfile(s) for s in source)):
        for s in source:
            yield from _iter_blocks(s, chunk)
        return
    if hasattr(source, "read"):
        while True:
            b = source.read(chunk)
            if not b:
                return
            yield b.encode() if isinstance(b, str) else b
        return
    buf = io.BytesIO()
    for line in source:  # iterable of lines (e.g. a subprocess stdout)
        buf.write(line.encode() if isinstance(line, str) else line)
        if buf.tell() >= chunk:
            yield buf.getvalue()
            buf = io.BytesIO()
    if buf.tell():
        yield buf.getvalue()


class PairBinner:
    """Device pair binner for one genome (owns an ``hh_binner``)."""

    def __init__(self, genome: dict, chroms, stream=None):
        _lib.require_gpu()
        self.genome = dict(genome)
        self.chroms = chroms
        self.order, names, codes, policy = _name_table(self.genome, chroms)
        self.n = len(self.order)
        blob = b"".join(n.encode() + b"\0" for n in names)
        ids = np.asarray(codes, dtype=np.int32)
        h = C.c_void_p()
        call("hh_binner_create", self.n, blob, ptr(ids), len(names), policy, C.byref(h))
        self._h = h
        self.stream = stream
        self.targets: list[Target] = []
        self.finished = False

    def add_target(self, res: int, local: bool = False, haplotype: bool = False) -> Target:
        res = int(res)
        nb = np.array([self.genome[c] // res + 1 for c in self.order], dtype=np.int64)
        first = np.concatenate([[0], np.cumsum(nb)[:-1]]).astype(np.int64) if self.n else np.zeros(0, np.int64)
        total = int(nb.sum())
        if haplotype:
            start = np.concatenate([first, first + total])
            n_bins = 2 * total
        else:
            start = np.concatenate([first, first])  # the P half is never selected
            n_bins = total
        if n_bins == 0:
            raise ValueError("empty genome")
        idx = C.c_int32(-1)
        call("hh_binner_add_target", self._h, res, int(bool(local)), ptr(np.ascontiguousarray(start)),
             ptr(nb.astype(np.int32)), int(n_bins), C.byref(idx))
        t = Target(res, bool(local), bool(haplotype), idx.value)
        t.n_bins = n_bins
        t.chrom_first = first
        t.chrom_nbins = nb
        self.targets.append(t)
        return t

    def add_impute_target(self, res: int, local: bool, unimputed=None, L: int = 0, imin: int = 2,
                          ratio: float = 0.9) -> Target:
        """An imputation target (haplotype layout, ordered cells); whole
        targets take the dense unimputed whole matrix at this resolution."""
        res = int(res)
        nb = np.array([self.genome[c] // res + 1 for c in self.order], dtype=np.int64)
        first = np.concatenate([[0], np.cumsum(nb)[:-1]]).astype(np.int64)
        total = int(nb.sum())
        start = np.concatenate([first, first + total])
        n_bins = 2 * total
        um = None
        if not local:
            um = np.ascontiguousarray(unimputed, dtype=np.int64)
            if um.shape != (n_bins, n_bins):
                raise ValueError(f"unimputed matrix must be {n_bins} x {n_bins}")
        idx = C.c_int32(-1)
        call("hh_binner_add_impute_target", self._h, res, int(bool(local)), ptr(start), ptr(nb.astype(np.int32)),
             n_bins, ptr(um), int(L), int(imin), float(ratio), C.byref(idx))
        t = Target(res, bool(local), True, idx.value)
        t.n_bins, t.chrom_first, t.chrom_nbins = n_bins, first, nb
        self.targets.append(t)
        return t

    def last_reached(self):
        """(byte offset in the fed stream, target index) of the last M-pass
        line that reached the imputation neighbourhood step, or (-1, -1)."""
        off, t = C.c_int64(0), C.c_int32(0)
        call("hh_binner_last_reached", self._h, C.byref(off), C.byref(t))
        return int(off.value), int(t.value)

    def set_stale(self, t: Target, pp_sum: int, ok: bool):
        call("hh_binner_set_stale", self._h, t.index, int(pp_sum), int(bool(ok)))

    def feed(self, source, fmt: PairsFormat, chunk_bytes: int = CHUNK_BYTES):
        """Parse + bin a pair source (see _iter_blocks); lines are split at
        newlines across blocks and files exactly like `cat file1 file2 |`."""
        carry = b""
        for block in _iter_blocks(source, chunk_bytes):
            data = carry + block if carry else block
            cut = data.rfind(b"\n") + 1
            if cut:
                self._feed_bytes(data[:cut], fmt, chunk_bytes)
            carry = data[cut:]
        if carry:
            self._feed_bytes(carry, fmt, chunk_bytes)

    def _feed_bytes(self, data: bytes, fmt, chunk_bytes):
        call("hh_binner_feed", self._h, data, len(data), C.byref(fmt), int(chunk_bytes), self.stream)

    def feed_device(self, ptr_dev: int, nbytes: int, fmt: PairsFormat):
        call("hh_binner_feed_device", self._h, C.c_void_p(ptr_dev), int(nbytes), C.byref(fmt), self.stream)

    def stats(self) -> dict:
        v = np.zeros(4, np.int64)
        call("hh_binner_stats", self._h, ptr(v))
        return dict(lines=int(v[0]), binned=int(v[1]), skipped_chrom=int(v[2]), skipped_mark=int(v[3]))

    def finish(self):
        call("hh_binner_finish", self._h, self.stream)
        self.finished = True

    def n_pairs(self, t: Target) -> int:
        return self.sizes(t)[1]

    def sizes(self, t: Target):
        """(pixels, pairs) of a target (pixels = -1 before finish)."""
        a, b = C.c_int64(0), C.c_int64(0)
        call("hh_binner_target_nnz", self._h, t.index, C.byref(a), C.byref(b))
        return int(a.value), int(b.value)

    def pixels(self, t: Target):
        """(bin1, bin2, count) int32 host arrays of a finished target, sorted
        by (bin1, bin2), bin1 <= bin2, global bin ids of the target layout."""
        if not self.finished:
            self.finish()
        nnz, npairs = C.c_int64(0), C.c_int64(0)
        call("hh_binner_target_nnz", self._h, t.index, C.byref(nnz), C.byref(npairs))
        n = int(nnz.value)
        b1, b2, c = (np.empty(n, np.int32) for _ in range(3))
        call("hh_binner_download", self._h, t.index, ptr(b1), ptr(b2), ptr(c))
        return b1, b2, c

    def pixels_device(self, t: Target):
        """(bin1_ptr, bin2_ptr, count_ptr, nnz): device pointers of a finished
        target's int32 pixel table (valid until close())."""
        if not self.finished:
            self.finish()
        nnz, npairs = C.c_int64(0), C.c_int64(0)
        call("hh_binner_target_nnz", self._h, t.index, C.byref(nnz), C.byref(npairs))
        p1, p2, pc = C.c_void_p(), C.c_void_p(), C.c_void_p()
        call("hh_binner_pixels_device", self._h, t.index, C.byref(p1), C.byref(p2), C.byref(pc))
        return p1.value or 0, p2.value or 0, pc.value or 0, int(nnz.value)

    def chrom_offsets(self, t: Target) -> np.ndarray:
        """cooler ``indexes/chrom_offset`` of a target's bin layout (haplotype:
        the M chromosomes then the P chromosomes)."""
        nb = np.asarray(t.chrom_nbins, dtype=np.int64)
        if t.haplotype:
            nb = np.concatenate([nb, nb])
        return np.concatenate([[0], np.cumsum(nb)]).astype(np.int64)

    def contact_matrix(self, t: Target, ignore_diags=1, cis_only=None, row_range=None):
        """The target's pixel table straight into an HBM-resident
        ``ice.ContactMatrix`` (no host round trip): bin -> cooler -> balance
        of TraditionalMatrixConstruction (matrixBuilding.py:617-714) without
        the cooler file.  ``cis_only`` defaults to the target being local
        (HiCHap balances localRes coolers with --cis-only, :713)."""
        from .ice import ContactMatrix
        p1, p2, pc, nnz = self.pixels_device(t)
        cis = t.local if cis_only is None else bool(cis_only)
        return ContactMatrix.from_device_pixels(p1, p2, pc, t.n_bins, self.chrom_offsets(t), ignore_diags, cis,
                                                row_range=row_range, stream=self.stream, nnz=nnz)

    def close(self):
        if getattr(self, "_h", None):
            call("hh_binner_free", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def neighborhood_index(L):
    """GetNeighborhoodIndex (matrixBuilding.py:721-732): the disc around
    (L+1, L+1) -- not the window centre -- of radius sqrt(L)."""
    import math
    center = L + 1
    ii, jj = [], []
    for i in range(L * 2 + 1):
        for j in range(L * 2 + 1):
            if math.sqrt((i - center) ** 2 + (j - center) ** 2) < math.sqrt(L):
                ii.append(i)
                jj.append(j)
    return ii, jj


def line_at(source, offset):
    """The text line starting at `offset` of a source's `cat` stream (bytes,
    a path or a list of paths)."""
    if isinstance(source, (bytes, bytearray, memoryview)):
        b = bytes(source)
        e = b.find(b"\n", offset)
        return b[offset:] if e < 0 else b[offset:e]
    paths = [source] if isinstance(source, (str, os.PathLike)) else list(source)
    out = b""
    for p in paths:
        size = os.path.getsize(p)
        if offset >= size and not out:
            offset -= size
            continue
        with open(p, "rb") as f:
            f.seek(offset)
            chunk = f.readline()
        out += chunk
        offset = 0
        if chunk.endswith(b"\n"):
            break
    return out.rstrip(b"\n")


# ------------------------------------------------------ reference shapes
S_DTYPE = np.dtype({"names": ["bin1", "bin2", "IF"], "formats": [np.int64, np.int64, np.float64]})


def _sparse(x, y, v):
    out = np.zeros(len(v), dtype=S_DTYPE)
    out["bin1"] = x
    out["bin2"] = y
    out["IF"] = v
    return out


def whole_sparse_dict(b1, b2, cnt, bins: dict):
    """WholeMatrixToSparseDict (:457-505) from a global pixel table: intra
    blocks (upper triangle) keyed by chrom, inter blocks (i < j in
    Sort_Chromosomes order, full block) keyed 'c1_c2'; local bin ids."""
    order = sort_chromosomes(bins)
    starts = np.array([bins[c][0] for c in order], dtype=np.int64)
    ends = np.array([bins[c][1] + 1 for c in order], dtype=np.int64)
    b1 = np.asarray(b1, np.int64)
    b2 = np.asarray(b2, np.int64)
    cnt = np.asarray(cnt)
    out = {}
    row_lo = np.searchsorted(b1, starts, "left")
    row_hi = np.searchsorted(b1, ends, "left")
    for i, c1 in enumerate(order):
        sl = slice(row_lo[i], row_hi[i])
        x, y, v = b1[sl], b2[sl], cnt[sl]
        cj = np.searchsorted(ends, y, "right")  # chromosome of bin2
        o = np.argsort(cj, kind="stable")       # blocks in order, rows/cols kept row-major
        x, y, v, cj = x[o], y[o], v[o], cj[o]
        bounds = np.searchsorted(cj, np.arange(len(order) + 1), "left")
        for j in range(i, len(order)):
            s = slice(bounds[j], bounds[j + 1])
            blk = _sparse(x[s] - starts[i], y[s] - starts[j], v[s].astype(np.float64))
            if j == i:
                out[c1] = blk
            elif i != len(order) - 1:
                out[c1 + "_" + order[j]] = blk
    return out


def local_sparse_dict(b1, b2, cnt, t: Target, order, prefix=""):
    """IntraMatrixToSparseDict (:508-525) from a local target's pixel table:
    {prefix + chrom: upper-triangle pixels in chromosome-local bins}."""
    b1 = np.asarray(b1, np.int64)
    b2 = np.asarray(b2, np.int64)
    half = 1 if prefix == "P" else 0
    out = {}
    for k, c in enumerate(order):
        s0 = int(t.chrom_first[k]) + (half * int(t.chrom_nbins.sum()) if t.haplotype else 0)
        s1 = s0 + int(t.chrom_nbins[k])
        lo, hi = np.searchsorted(b1, [s0, s1], "left")
        out[prefix + c] = _sparse(b1[lo:hi] - s0, b2[lo:hi] - s0, np.asarray(cnt[lo:hi], np.float64))
    return out


def dense_from_pixels(b1, b2, cnt, n, offset=0):
    """Symmetric dense int64 n x n from upper-triangle pixels (the reference's
    dense matrices, :554, :567-570); rows/cols shifted by ``offset``."""
    M = np.zeros((n, n), dtype=np.int64)
    i = np.asarray(b1, np.int64) - offset
    j = np.asarray(b2, np.int64) - offset
    c = np.asarray(cnt, np.int64)
    M[i, j] = c
    M[j, i] = c
    return M


__all__ = ["PairBinner", "PairsFormat", "pairs_format", "VALID_BED", "ALLELIC_BED", "load_genome",
           "sort_chromosomes", "chrom_bins", "haplotype_bins", "whole_sparse_dict", "local_sparse_dict",
           "dense_from_pixels", "strip_chr", "Target"]
