"""StructureFind numeric cores on MI355X — same class / method names and
arguments as ``HiCHap/StructureFind.py``:

* ``Distance_Decay(M, G_array)``          StructureFind.py:201-271
* ``Get_PCA(distance_bin, M, NG_array, SA)`` :302-342 (SA: Sliding_Approach :274-299)
* ``Select_PC_new(Cor_M, OE_M, pca)``      :374-423
* ``Select_Allelic_PC(pcs, trad_pc)``      :446-460
* ``Get_Gap(M)`` / ``Get_DI(M, Gap, w)``   :721-751 / :804-839
* ``Gap_Filter(Gap, M)``                   :753-802
* ``Data_preprocess`` / ``viterbipath`` / ``BoundaryCall`` /
  ``BoundaryFilter`` / ``BoundaryToDomain``  :842-1342 (``tads.py``)

The O(N^2) / O(N^2 n) work (column nonzeros, per-distance sums, O/E,
Pearson correlation on fp64 MFMA, top-3 PCA, the masked sums of the PC
selection, the windowed DI statistics) runs in HIP kernels; O(N) decisions
(gap thresholds, bin counts, the selection rules) are host glue written with
the reference's own NumPy expressions.  ``Get_PCA`` returns the correlation
and O/E matrices as lazy device-backed arrays (``np.asarray`` materialises
them) so the N x N products stay in HBM for ``Select_PC_new``.
"""
from __future__ import annotations

import ctypes as C
import warnings

import numpy as np

from . import _lib
from ._lib import call, ptr
from .tads import GaussianMixtureHMM, TADCalling  # noqa: F401  (TAD HMM + boundary rules)

PCA_TOL = 1e-13   # max entry change of the unit Ritz vectors between iterations
PCA_MAX_ITERS = 2000


def py2_float_str(v):
    """Python 2 ``str(float)``: '%.12g', with '.0' on integral values."""
    t = "%.12g" % float(v)
    return t + ".0" if t.lstrip("-").isdigit() else t


class _Comp:
    """Owns an ``hh_comp*`` (one chromosome's matrix in HBM)."""

    def __init__(self, M, stream=None):
        _lib.require_gpu()
        self.stream = stream  # HIP stream handle (int / c_void_p) or None = default
        self._dev = None
        self._host = None
        if getattr(M, "is_cuda", False):  # a device-resident torch tensor: no copy
            import torch
            if M.dtype != torch.float64 or M.dim() != 2 or M.shape[0] != M.shape[1] or not M.is_contiguous():
                raise ValueError("expected a contiguous square float64 device tensor")
            self._dev = M
            self.N = int(M.shape[0])
            src, on_dev = C.c_void_p(M.data_ptr()), 1
        else:
            self._host = np.ascontiguousarray(M, dtype=np.float64)
            if self._host.ndim != 2 or self._host.shape[0] != self._host.shape[1]:
                raise ValueError("expected a square matrix")
            self.N = self._host.shape[0]
            src, on_dev = ptr(self._host), 0
        h = C.c_void_p()
        call("hh_comp_create", src, self.N, on_dev, self._s(), C.byref(h))
        self.h = h
        self.decline = None
        self.NG = None
        self.sa = False
        self._sa_host = None

    def _s(self):
        return None if self.stream is None else C.c_void_p(int(self.stream))

    @property
    def M(self):
        if self._host is None:
            self._host = self._dev.cpu().numpy()
        return self._host

    def colnnz(self):
        out = np.empty(self.N, np.int64)
        call("hh_comp_colnnz", self.h, ptr(out), self._s())
        return out

    def diag_sums(self, gap_mask):
        g = np.ascontiguousarray(gap_mask, dtype=np.uint8)
        out = np.empty(self.N, np.float64)
        call("hh_comp_diag_sums", self.h, ptr(g), ptr(out), self._s())
        return out

    def sliding_oe(self, decline, step):
        """Sliding_Approach O/E on the device (None: back to the plain O/E)."""
        if decline is None:
            call("hh_comp_sliding_oe", self.h, None, 0, self._s())
            self.sa = False
            return
        self.decline = np.ascontiguousarray(decline, dtype=np.float64)
        call("hh_comp_sliding_oe", self.h, ptr(self.decline), int(step), self._s())
        self.sa = True
        self._sa_host = None

    def sa_matrix(self):
        if self._sa_host is None:
            self._sa_host = np.empty((self.N, self.N), np.float64)
            call("hh_comp_get_sliding_oe", self.h, ptr(self._sa_host), self._s())
        return self._sa_host

    def correlation(self, decline, NG):
        self.decline = np.ascontiguousarray(decline, dtype=np.float64)
        self.NG = np.ascontiguousarray(NG, dtype=np.int64)
        call("hh_comp_correlation", self.h, ptr(self.decline), ptr(self.NG), self.NG.size, self._s())

    def cor(self):
        n = self.NG.size
        out = np.empty((n, n), np.float64)
        call("hh_comp_get_cor", self.h, ptr(out), self._s())
        return out

    def pca(self, k=3):
        """Top-k PCA components of the correlation (block Krylov on the
        device, hh_comp_pca).  Warns (RuntimeWarning) when the eigensolver
        stopped at its product budget without meeting PCA_TOL; the status is
        kept in ``self.pca_status``."""
        n = self.NG.size
        comps = np.empty((k, n), np.float64)
        ev = np.empty(k, np.float64)
        it = C.c_int32(0)
        call("hh_comp_pca", self.h, int(k), PCA_TOL, PCA_MAX_ITERS, ptr(comps), ptr(ev), C.byref(it), self._s())
        conv, prods, cyc, meth = (C.c_int32(0) for _ in range(4))
        call("hh_comp_pca_status", self.h, C.byref(conv), C.byref(prods), C.byref(cyc), C.byref(meth))
        self.pca_status = {"converged": bool(conv.value), "products": prods.value, "cycles": cyc.value,
                           "method": "krylov" if meth.value in (1, 2) else "subspace", "eigvals": ev.copy(),
                           # the one-launch orthogonalisation's grid could not become co-resident and the
                           # solve was redone on the multi-launch path (hh_comp_pca)
                           "ortho_fallback": meth.value == 2}
        if not conv.value:
            warnings.warn(f"compartment PCA did not converge to {PCA_TOL:g} within its budget "
                          f"({prods.value} correlation products, {self.pca_status['method']}); "
                          f"the top eigenvalues may be (nearly) degenerate", RuntimeWarning, stacklevel=3)
        return comps, ev, it.value

    def select_stats(self, pcs, eps=1e-5):
        p = np.ascontiguousarray(pcs, dtype=np.float64)
        k = p.shape[0]
        st = np.empty((k, 8), np.float64)
        call("hh_comp_select_stats", self.h, ptr(p), int(k), float(eps), ptr(st), self._s())
        return st

    def __del__(self):
        try:
            if self.h:
                call("hh_comp_free", self.h)
                self.h = None
        except Exception:
            pass


class DeviceCorrelation:
    """Lazy n x n correlation matrix held in HBM (``np.asarray`` downloads)."""

    def __init__(self, comp: _Comp):
        self._c = comp
        self.shape = (comp.NG.size, comp.NG.size)
        self._host = None

    def __array__(self, dtype=None, copy=None):
        if self._host is None:
            self._host = self._c.cor()
        return self._host if dtype is None else self._host.astype(dtype)


class DeviceOE:
    """Lazy O/E matrix ``OE[:, NG]`` (N x n); ``[NG]`` gives the NG rows, the
    form Select_PC_new receives (StructureFind.py:519)."""

    def __init__(self, comp: _Comp, rows=None):
        self._c = comp
        self._rows = rows
        n = comp.NG.size
        self.shape = (comp.N if rows is None else len(rows), n)

    def __getitem__(self, idx):
        rows = np.arange(self._c.N)[idx] if self._rows is None else np.asarray(self._rows)[idx]
        return DeviceOE(self._c, np.asarray(rows, dtype=np.int64))

    def __array__(self, dtype=None, copy=None):
        c = self._c
        rows = np.arange(c.N) if self._rows is None else self._rows
        if c.sa:
            out = c.sa_matrix()[np.ix_(rows, c.NG)]
            return out if dtype is None else out.astype(dtype)
        sub = c.M[np.ix_(rows, c.NG)]
        d = np.abs(rows[:, None] - c.NG[None, :])
        out = np.zeros_like(sub)
        nz = sub != 0
        out[nz] = sub[nz] / c.decline[d[nz]]
        return out if dtype is None else out.astype(dtype)


class _ThunkDict(dict):
    """{chrom: matrix} whose values are made by a thunk on first access."""

    def __init__(self):
        super().__init__()
        self._thunks = {}

    def put(self, key, thunk):
        self._thunks[key] = thunk

    def __getitem__(self, key):
        if not dict.__contains__(self, key):
            if key not in self._thunks:
                raise KeyError(key)
            dict.__setitem__(self, key, self._thunks.pop(key)())
        return dict.__getitem__(self, key)

    def __contains__(self, key):
        return dict.__contains__(self, key) or key in self._thunks

    def keys(self):
        return list(dict.keys(self)) + [k for k in self._thunks if not dict.__contains__(self, k)]

    def __iter__(self):
        return iter(self.keys())

    def __len__(self):
        return len(self.keys())

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def values(self):
        return [self[k] for k in self.keys()]


class StructureFind(TADCalling):
    """Numeric part of HiCHap's StructureFind (StructureFind.py:27); the TAD
    HMM / boundary-rule methods come from ``tads.TADCalling``."""

    def __init__(self, cooler_fil=None, Res=40000, Allelic=False, GapFile=None, Loop_ratio=0.6,
                 Loop_strength=16, stream=None):
        self.cooler_fil = "{}::{}".format(cooler_fil, Res) if cooler_fil else None
        self.Res = Res
        self.Allelic = Allelic
        self.Gap_file = GapFile
        self.ratio = Loop_ratio
        self.LoopStrength = Loop_strength
        self._comp = None
        self._comp_src = None
        self.stream = stream  # HIP stream for the device calls (None = default stream)

    # ------------------------------------------------------ compartments
    def Distance_Decay(self, M, G_array):
        """Distance-decay expected counts (StructureFind.py:201-271).
        Returns (distance_bin, G_array, NG_array)."""
        comp = _Comp(M, self.stream)
        self._comp, self._comp_src = comp, M
        size = comp.N
        bin_arange = np.arange(size)
        if G_array is None:
            nonzero_mask = comp.colnnz() / float(size)
            gap_mask = np.where(nonzero_mask <= 0.05, True, False)
            G_array = bin_arange[gap_mask]
            NG_array = bin_arange[~gap_mask]
        else:
            G_array = np.asarray(G_array)
            gap_mask = np.zeros(size, dtype=bool)
            gap_mask[G_array.astype(np.int64)] = True
            NG_array = bin_arange[~gap_mask]
        distance_bin = comp.diag_sums(gap_mask)
        # bin counts per distance (the reference's loop :252-268, vectorised)
        Gs = np.sort(np.asarray(G_array, dtype=np.int64))
        dd = np.arange(size)
        gap_num = (np.searchsorted(Gs, size - 1 - dd, side="right")
                   + (Gs.size - np.searchsorted(Gs, dd, side="left")))
        bin_num = np.asarray((size - dd), dtype=float) * 2 - gap_num
        bin_num[0] = float(size - 0) - np.sum((0 <= Gs) & (Gs <= size - 1))
        ok = bin_num > 0
        distance_bin[ok] = distance_bin[ok] / bin_num[ok]
        return distance_bin, G_array, NG_array

    def Get_PCA(self, distance_bin, M, NG_array, SA=False):
        """O/E, Pearson correlation and top-3 PCA (StructureFind.py:302-342).
        Returns (pca_components[3 x n], Cor (lazy), OE[:, NG] (lazy)).
        ``SA=True`` uses the Sliding_Approach O/E (:274-299, window 600 kb)."""
        comp = self._comp if (self._comp is not None and self._comp_src is M) else None
        if comp is None:
            comp = _Comp(M, self.stream)
            self._comp, self._comp_src = comp, M
        decline = distance_bin
        decline[decline == 0] = decline[np.nonzero(decline)].min()
        if SA:
            step = 600000 // self.Res // 2
            if step < 1:  # the reference reads decline[N], decline[N + 1] here
                raise IndexError(f"Sliding_Approach window 600000 // Res {self.Res} // 2 = 0 bins")
            comp.sliding_oe(decline, step)
        elif comp.sa:
            comp.sliding_oe(None, 0)
        comp.correlation(decline, NG_array)
        pcs, _, _ = comp.pca(3)
        self.pca_status = comp.pca_status
        return pcs, DeviceCorrelation(comp), DeviceOE(comp)

    def Select_PC_new(self, Cor_M, OE_M, pca):
        """PC choice and A/B sign (StructureFind.py:374-423)."""
        pca = np.asarray(pca)
        if isinstance(Cor_M, DeviceCorrelation):
            comp = Cor_M._c
        else:
            comp = _array_comp(np.asarray(Cor_M), np.asarray(OE_M))
        st = comp.select_stats(pca[:3])
        nums, values = 0, 0
        for i in range(len(pca)):
            minus = _means_minus(st[i], pca[i])
            if minus > values:
                values, nums = minus, i
        pc = pca[nums]
        with np.errstate(invalid="ignore", divide="ignore"):
            values_a = st[nums, 4] / st[nums, 5]
            values_b = st[nums, 6] / st[nums, 7]
        if values_b > values_a:
            pc = pc.copy() * -1
        return pc

    def Select_Allelic_PC(self, pca_components, Tranditional_PC, eps=0.7):
        """Supervised PC choice for haplotype data (StructureFind.py:446-460)."""
        PCC = [abs(np.corrcoef(pc, Tranditional_PC)[0][1]) for pc in pca_components]
        if np.max(PCC) < eps:
            print("    PCC too low for this chromosome, check it if possible!")
        return pca_components[int(np.argmax(PCC))]

    def compartment(self, M, Tranditional_PC=None):
        """Per-chromosome body of Compartment() (StructureFind.py:509-527):
        the selected PC at full length (zeros at gap bins)."""
        if not getattr(M, "is_cuda", False):
            M = np.asarray(M, dtype=np.float64)
        distance_bin, Gap, NonGap = self.Distance_Decay(M=M, G_array=None)
        pca, Cor_M, OE_M = self.Get_PCA(distance_bin=distance_bin, M=M, NG_array=NonGap)
        out = np.zeros((M.shape[0],), dtype=float)
        if Tranditional_PC is None:
            out[NonGap] = self.Select_PC_new(Cor_M, OE_M[NonGap], pca)
        else:
            raw = np.zeros((len(pca), M.shape[0]))
            raw[:, NonGap] = pca
            out[NonGap] = self.Select_Allelic_PC(raw, Tranditional_PC)[NonGap]
        return out


    # ------------------------------------------------- cooler-driven steps
    def _chroms_and_matrices(self, balance_traditional):
        """The per-chromosome dense matrices the reference fetches from its
        cooler (StructureFind.py:499-513, :848-865): traditional data with
        ``balance_traditional`` (NaN -> 0 when balanced), haplotype data raw,
        chromosomes filtered by the Allelic prefix."""
        from .coolio import Cooler
        if not self.cooler_fil:
            raise ValueError("no cooler file (StructureFind(cooler_fil=..., Res=...))")
        with Cooler(self.cooler_fil) as c:
            if self.Allelic is False:
                chroms = list(c.chromnames)
            elif self.Allelic in ("Maternal", "Paternal"):
                chroms = [x for x in c.chromnames if x.startswith(self.Allelic[0])]
            else:
                raise ValueError(f"Unknown key word {self.Allelic}, only Maternal, Paternal, False allowed")
            bal = balance_traditional and self.Allelic is False
            out = {}
            for chro in chroms:
                M = c.matrix(balance=bal).fetch(chro)
                out[chro] = np.nan_to_num(M) if bal else M
        return chroms, out

    @staticmethod
    def Loading_Tranditional_PC(fil):
        """``chrom value`` lines -> {chrom: PC array} (StructureFind.py:426-443)."""
        d = {}
        with open(fil) as f:
            for line in f:
                parts = line.split()
                if parts:
                    d.setdefault(parts[0], []).append(parts[-1])
        return {k: np.array(v, dtype=float) for k, v in d.items()}

    def _gaps(self):
        """The haplotype gap lists (CallPeaks :1985-1991): ``GapFile`` as a
        dict {str(Res): {chrom: gap}} / {chrom: gap}, or an .npz path read
        without unpickling (a pickled npz raises: pass the dict)."""
        G = self.Gap_file
        if G is None:
            raise ValueError("Gap file needed for haplotype-resolved loop calling ...")
        if isinstance(G, (str, bytes)):
            with np.load(G, allow_pickle=False) as z:
                G = {k: z[k] for k in z.files}
        if str(self.Res) in G:
            G = G[str(self.Res)]
            G = G[()] if hasattr(G, "shape") and G.shape == () else G
        return G

    def CallPeaks(self, outfil, Allelic=False):
        """HICCUPS loop calling from the cooler (StructureFind.py:1954-2043):
        raw, balanced and weight read from ``cooler_fil::Res`` itself
        (:2006-2010) as pixel bands -- no dense N x N -- then
        hichap_master_amd.loops on the GPU; writes the reference's file."""
        from . import loops
        gaps = None if Allelic is False else self._gaps()
        out = loops.call_peaks_cooler(self.cooler_fil, outfil, self.Res, Allelic, gaps)
        self.chroms = list(out)
        return out

    def Compartment(self, SA=False, Tranditional_PC_file=None, Matrix_Dict=None):
        """Compartment() (StructureFind.py:491-554): raw matrices from the
        cooler (or ``Matrix_Dict``), one selected PC per chromosome in
        ``Compartment_Dict`` (zeros at gap bins); haplotype data also keep
        the three raw PCs in ``RawPCA``.  From a cooler file each
        chromosome's raw matrix is built on the GPU from its pixels
        (:499-513 fetch densely on the host: N^2 x 8 B through PCIe; here
        only the pixel table crosses), ``Matrix_Dict`` a lazy dense view."""
        from_file = Matrix_Dict is None
        if from_file:
            chroms = self._cooler_chroms()
            from .tads import _LazyMatrices
            Matrix_Dict = _LazyMatrices(self.cooler_fil, chroms, False)
        else:
            chroms = list(Matrix_Dict)
        trad = self.Loading_Tranditional_PC(Tranditional_PC_file) if self.Allelic is not False else None
        self.chroms, self.Matrix_Dict = chroms, Matrix_Dict
        self.Compartment_Dict, self.RawPCA = {}, {}
        # the gap-refilled O/E and correlation matrices (:550-554), made on
        # first access from the device-held ones (Plot_Compartment reads them)
        self.Cor_Martrix_Dict, self.OE_Matrix_Dict = _ThunkDict(), _ThunkDict()
        for chro in chroms:
            if from_file:
                M = self._device_raw_matrix(chro)
                M_host = (lambda chro=chro: np.asarray(Matrix_Dict[chro], dtype=np.float64))
            else:
                M = np.asarray(Matrix_Dict[chro], dtype=np.float64)
                M_host = M
            distance_bin, Gap, NonGap = self.Distance_Decay(M=M, G_array=None)
            pca, Cor_M, OE_M = self.Get_PCA(distance_bin=distance_bin, M=M, NG_array=NonGap, SA=SA)
            out = np.zeros(M.shape[0], dtype=float)
            if self.Allelic is False:
                out[NonGap] = self.Select_PC_new(Cor_M, OE_M[NonGap], pca)
            else:
                raw = np.zeros((len(pca), M.shape[0]))
                raw[:, NonGap] = pca
                self.RawPCA[chro] = raw
                out[NonGap] = self.Select_Allelic_PC(raw, trad[chro[1:]])[NonGap]
            self.Compartment_Dict[chro] = out
            # thunks over host inputs only (M, decline, NonGap): this
            # chromosome's device state (matrix, correlation, Krylov
            # workspace) is freed now, not kept alive by the dicts
            dec = np.array(distance_bin, dtype=np.float64)
            for d, kind in ((self.OE_Matrix_Dict, "OE"), (self.Cor_Martrix_Dict, "Cor")):
                d.put(chro, self._refill_thunk(M_host, dec, NonGap, SA, kind))
            del Cor_M, OE_M, M
            self._comp = self._comp_src = None
        return self.Compartment_Dict

    def _cooler_chroms(self):
        """The chromosomes the reference's Compartment reads (:499-506)."""
        from .coolio import Cooler
        if not self.cooler_fil:
            raise ValueError("no cooler file (StructureFind(cooler_fil=..., Res=...))")
        with Cooler(self.cooler_fil) as c:
            if self.Allelic is False:
                return list(c.chromnames)
            if self.Allelic in ("Maternal", "Paternal"):
                return [x for x in c.chromnames if x.startswith(self.Allelic[0])]
        raise ValueError(f"Unknown key word {self.Allelic}, only Maternal, Paternal, False allowed")

    def _device_raw_matrix(self, chro):
        """``cooler.matrix(balance=False).fetch(chro)`` as a float64 device
        tensor built from the chromosome's pixels (hh_dense_from_cells:
        symmetric scatter of the upper-triangle cells, exact int64, then one
        conversion pass)."""
        import torch
        from .coolio import Cooler
        from .matrixBuilding import dense_from_cells_device
        with Cooler(self.cooler_fil) as c:
            lo, hi = c.extent(chro)
            b1, b2, v = c.pixel_rows(lo, hi)
        keep = b2 < hi
        D = dense_from_cells_device((b1[keep], b2[keep], v[keep]), hi - lo, lo, symmetric=True,
                                    stream=None if self.stream is None else C.c_void_p(int(self.stream)))
        return D.to(torch.float64)

    def _refill_thunk(self, M, decline, NonGap, SA, kind):
        """Refill_Gap(M, OE or Cor) made on first access from the host inputs
        (``M`` an array or a zero-argument function giving it): the
        correlation (and the Sliding_Approach O/E) recomputed on the GPU in a
        short-lived hh_comp, the plain O/E on the host."""
        def make():
            nonlocal M
            if callable(M):
                M = M()
            NG = np.asarray(NonGap, dtype=np.int64)
            if kind == "OE" and not SA:
                sub = M[:, NG]
                d = np.abs(np.arange(M.shape[0])[:, None] - NG[None, :])
                X = np.zeros_like(sub)
                nz = sub != 0
                X[nz] = sub[nz] / decline[d[nz]]
                return self.Refill_Gap(M, X, NG, "OE")
            comp = _Comp(M, self.stream)
            try:
                if SA:
                    comp.sliding_oe(decline, 600000 // self.Res // 2)
                comp.correlation(decline, NG)
                X = np.asarray(DeviceCorrelation(comp) if kind == "Cor" else DeviceOE(comp))
            finally:
                call("hh_comp_free", comp.h)
                comp.h = None
            return self.Refill_Gap(M, X, NG, kind)
        return make

    def Refill_Gap(self, M1, M2, NonGap, dtype):
        """Refill_Gap (StructureFind.py:463-488): the n x n correlation or the
        N x n O/E columns back at the non-gap positions of an N x N zero
        matrix.  'Cor': R[NG[i], NG[j]] = M2[j][i].  'OE': the reference
        transposes its output inside the loop (:483-486), so row and column
        writes alternate (row NG[0], column NG[1], row NG[2], ...; later writes
        win) and the result is transposed when len(NonGap) is odd -- kept as
        is, since Plot_Compartment draws exactly that."""
        N = np.shape(M1)[0]
        NG = np.asarray(NonGap, dtype=np.int64)
        X = np.asarray(M2, dtype=np.float64)
        R = np.zeros((N, N), dtype=np.float64)
        if dtype == "Cor":
            R[np.ix_(NG, NG)] = X.T
        elif dtype == "OE":
            XT = X.T
            flip = False
            for i in range(len(NG)):
                if flip:
                    R[:, NG[i]] = XT[i]
                else:
                    R[NG[i], :] = XT[i]
                flip = not flip
            if flip:
                R = R.T
        return R

    def OutPut_PC_To_txt(self, out):
        """``chrom<TAB>value`` per bin (StructureFind.py:557-576; haplotype
        chromosomes without their M/P prefix), values as Python 2's
        ``str(float)`` prints them (12 significant digits)."""
        with open(out, "w") as f:
            for chro, pc in self.Compartment_Dict.items():
                name = chro if self.Allelic is False else chro[1:]
                for v in pc:
                    f.write(f"{name}\t{py2_float_str(v)}\n")

    # --------------------------------------------------------------- TADs
    def TAD_parameter_init(self, minTAD, maxTAD, state_num, window, test_type):
        """Prior parameters of the TAD scan (StructureFind.py:709-718)."""
        self.minTAD, self.maxTAD, self.state_num = minTAD, maxTAD, state_num
        self.window, self.test_type = window, test_type

    def Get_Gap(self, M):
        """Gap columns for TAD calling (StructureFind.py:721-751)."""
        _lib.require_gpu()
        lb = int(self.minTAD / self.Res)
        band = column_band(M, lb)
        N = band.shape[1]
        g = np.empty(N, np.uint8)
        call("hh_gap_scan", ptr(band), N, lb, lb, ptr(g), 0, None)
        return np.nonzero(g)[0]

    def Get_DI(self, M, Gap, window_bin):
        """Directionality index (StructureFind.py:804-839)."""
        _lib.require_gpu()
        N = np.shape(M)[0]
        g = np.zeros(N, np.uint8)
        g[np.asarray(Gap, dtype=np.int64)] = 1
        w = np.ascontiguousarray(np.broadcast_to(np.asarray(window_bin), (N,)), dtype=np.int32)
        if self.test_type not in ("ttest", "chitest"):
            return np.zeros(N)
        B = int(max(w.max(), 0))
        band = column_band(M, B)
        di = np.empty(N, np.float64)
        call("hh_di_scan", ptr(band), N, B, ptr(g), ptr(w), 0 if self.test_type == "ttest" else 1, ptr(di), 0,
             None)
        return di

    def Gap_Filter(self, Gap, M):
        """Gap runs kept for HMM training (StructureFind.py:753-802): runs of
        consecutive gap bins at least min(10, mean run length) long, plus the
        first and last bin."""
        Gap = np.asarray(Gap)
        if Gap.shape[0] <= 1:
            return []
        runs = []
        start = end = int(Gap[0])
        L = Gap.shape[0]
        for i in range(1, L):
            step = Gap[i] - Gap[i - 1] == 1
            if step and i == L - 1:
                end = int(Gap[i]) + 1
                runs.append((start, end))
            elif step:
                end = int(Gap[i]) + 1
            else:
                runs.append((start, end))
                start, end = int(Gap[i]), int(Gap[i]) + 1
        runs = sorted(set(runs))
        mean_len = np.mean([e - s for s, e in runs])
        kept = [r for r in runs if r[1] - r[0] >= min([10, mean_len])]
        out = []
        for s_, e_ in kept:
            out.extend(range(s_, e_))
        if 0 not in out:
            out.insert(0, 0)
        if np.shape(M)[0] - 1 not in out:
            out.append(np.shape(M)[0] - 1)
        return out

    def di_scan(self, M, window=None):
        """Data_preprocess's per-chromosome scan (:873-891): gap (with the
        first and last bin) and DI."""
        N = np.shape(M)[0]
        gap = list(self.Get_Gap(M))
        if 0 not in gap:
            gap.insert(0, 0)
        if N - 1 not in gap:
            gap.append(N - 1)
        gap = np.array(gap)
        wb = int((self.window if window is None else window) / self.Res)
        return gap, self.Get_DI(M, gap, np.ones(N, dtype=int) * wb)

    def di_scan_pixels(self, bin1, bin2, count, weight, lo, N, window=None):
        """``di_scan`` of one chromosome straight from cooler's pixel table
        (Data_preprocess :853-854 fetches the balanced dense matrix and
        applies np.nan_to_num; pass ``weight=None`` for the allelic
        ``balance=False`` path, :858-865): the band the scans read is built on
        the device, so the N x N matrix never exists.  ``bin1 <= bin2`` are
        global bin ids of unique pixels, the chromosome is bins [lo, lo + N).
        Returns (gap with the first / last bin, DI) like ``di_scan``."""
        _lib.require_gpu()
        b1 = np.ascontiguousarray(bin1, dtype=np.int64)
        b2 = np.ascontiguousarray(bin2, dtype=np.int64)
        c = np.ascontiguousarray(count, dtype=np.float64)
        if not (b1.shape == b2.shape == c.shape):
            raise ValueError("bin1, bin2 and count must have the same length")
        w = None if weight is None else np.ascontiguousarray(weight, dtype=np.float64)
        lb = int(self.minTAD / self.Res)
        wb = int((self.window if window is None else window) / self.Res)
        if self.test_type not in ("ttest", "chitest"):
            raise ValueError(f"unknown test type {self.test_type!r}")
        win = np.full(int(N), wb, dtype=np.int32)
        g = np.empty(int(N), np.uint8)
        di = np.empty(int(N), np.float64)
        call("hh_tad_scan_pixels", ptr(b1), ptr(b2), ptr(c), b1.size, None if w is None else ptr(w),
             0 if w is None else w.size, int(lo), int(N), lb, ptr(win), 0 if self.test_type == "ttest" else 1,
             ptr(g), ptr(di), 0, None)
        return np.nonzero(g)[0], di


def column_band(M, B):
    """band[B + k, j] = M[j + k, j] for k in [-B, B] (0 outside), diagonal-
    major ((2B+1) x N): the part of each column the gap / DI scans read, so
    N x N never crosses PCIe."""
    M = np.asarray(M)
    N = M.shape[0]
    band = np.zeros((2 * B + 1, N), dtype=np.float64)
    for k in range(-min(B, N - 1), min(B, N - 1) + 1):
        d = np.diagonal(M, offset=-k)  # M[t + k, t] (k >= 0) / M[t, t - k] (k < 0)
        if k >= 0:
            band[B + k, : N - k] = d
        else:
            band[B + k, -k:] = d
    return band


def _means_minus(st, pc):
    """means_minus (StructureFind.py:375-402) from the device sums."""
    loc = np.arange(len(pc))
    la, lb = loc[pc > 0], loc[pc < 0]
    if la.shape[0] == 0 or lb.shape[0] == 0:
        return 0
    size_a = la.max() - la.min()
    size_b = lb.max() - lb.min()
    lens = max(la.max(), lb.max()) - min(la.min(), lb.min())
    n_ab = st[3]
    mean_ab = st[2] / n_ab if n_ab else np.nan
    if n_ab == 0 or mean_ab == 0 or mean_ab == -1 or size_a <= lens / 2 or size_b <= lens / 2:
        return 0
    return st[0] / st[1] - mean_ab


def _array_comp(Cor, OE_ng):
    """Select_PC_new on host arrays: upload O/E[NG,NG] as the matrix with a
    unit decline and the given correlation."""
    n = Cor.shape[0]
    comp = _Comp(np.asarray(OE_ng, dtype=np.float64)[:, :n])
    comp.correlation(np.ones(n), np.arange(n))
    call("hh_comp_set_cor", comp.h, ptr(np.ascontiguousarray(Cor, dtype=np.float64)), None)
    return comp
