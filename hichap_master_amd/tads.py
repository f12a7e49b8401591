"""TAD calling after the DI scan — the HMM and boundary-rule half of
``HiCHap/StructureFind.py`` (Data_preprocess :842-915, init_parameter_state*
:918-1049, viterbipath :1113-1123, BoundaryMask :1126-1155, BoundaryCall
:1158-1188, modelPredict :1191-1209, Candidate_domains :1212-1229,
BoundaryFilter :1232-1268, BoundaryToDomain :1271-1342).

``TADCalling`` is mixed into ``StructureFind``; the methods keep the
reference's names, arguments and ``self`` attributes (``DI_all_train``,
``DI_dict``, ``Gap_all``, ``boundary_index``, ``boundary_filtered``,
``Domain_dict``).  Gap and DI come from the GPU scans (``Get_Gap`` /
``Get_DI``); the Viterbi dynamic program is host C++ behind the C-ABI
(``hh_viterbi_gmm``); the boundary rules are host NumPy.

Not built: ghmm's Baum-Welch training (``updateParameter`` / ``modelTrain``,
:1052-1110).  ghmm is a third-party C library absent here, its EM stopping
rule is unpinnable, and the reference trains on shuffled sequences
(``random.shuffle``, :1058-1063), so its trained model is not reproducible
anyway.  A model is supplied instead: ``GaussianMixtureHMM(A, B, pi)`` with
ghmm's parameter layout (e.g. exported from a ghmm run, or the untrained
priors of ``init_parameter_state3/5/6``).

Py2 -> Py3: the reference's structured arrays hold byte strings ('>S5',
'>S1') compared with ``str`` literals, which Py2 treats as equal; here they are
unicode ('<U5', '<U1') so the comparisons keep the reference's meaning.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import call, ptr

STATE_DTYPE = [("boundary", np.int64), ("state", "<U5"), ("rely", np.float64), ("raw_state", "<U1")]
MASK_STR = {3: [("220", 2, 2), ("200", 1, 1), ("2221", 3, 3), ("1000", 1, 1)],
            5: [("40", 1, 1)]}


class GaussianMixtureHMM:
    """A continuous HMM with Gaussian-mixture emissions in ghmm's layout:
    ``A[i][j]`` transition, ``B[i] = [means, variances, weights]``, ``pi[i]``
    initial probabilities.  ``viterbi(seq)`` returns ``(path, log_p)`` like
    ghmm's ``model.viterbi(EmissionSequence)``; the getters mirror ghmm's."""

    def __init__(self, A, B, pi):
        self.A = np.ascontiguousarray(A, dtype=np.float64)
        B = [[np.asarray(b[0], float), np.asarray(b[1], float), np.asarray(b[2], float)] for b in B]
        self.mean = np.ascontiguousarray([b[0] for b in B], dtype=np.float64)
        self.var = np.ascontiguousarray([b[1] for b in B], dtype=np.float64)
        self.weight = np.ascontiguousarray([b[2] for b in B], dtype=np.float64)
        self.pi = np.ascontiguousarray(pi, dtype=np.float64)
        S, M = self.mean.shape
        if self.A.shape != (S, S) or self.pi.shape != (S,) or self.var.shape != (S, M) \
                or self.weight.shape != (S, M):
            raise ValueError("inconsistent HMM parameter shapes")

    @property
    def n_states(self):
        return self.mean.shape[0]

    def viterbi(self, seq):
        x = np.ascontiguousarray(seq, dtype=np.float64)
        S, M = self.mean.shape
        path = np.empty(x.size, np.int32)
        logp = C.c_double(0.0)
        call("hh_viterbi_gmm", ptr(x), x.size, S, M, ptr(self.A), ptr(self.pi), ptr(self.mean), ptr(self.var),
             ptr(self.weight), ptr(path), C.byref(logp))
        return [int(s) for s in path], logp.value

    def getTransition(self, i, j):
        return float(self.A[i, j])

    def getEmission(self, i, j):
        return float(self.mean[i, j]), float(self.var[i, j]), float(self.weight[i, j])

    def getInitial(self, i):
        return float(self.pi[i])


def _gmm_prior(state_means, num):
    """B of init_parameter_state*: three components per state, variance
    num / 2, weights 1/3 (StructureFind.py:940-954, :986-1001, :1028-1045)."""
    numdists = 3
    var = num / (numdists - 1)
    W = 1.0 / numdists
    return [[[off(i) * var for i in range(numdists)], [var] * numdists, [W] * numdists] for off in state_means]


class TADCalling:
    """HMM + boundary-rule half of the reference's TAD calling."""

    model = None

    # ------------------------------------------------------------ priors
    def init_parameter_state3(self):
        """StructureFind.py:918-956 (0 downstream, 1 no bias, 2 upstream)."""
        A = [[0.85, 0.15, 0.00], [0.05, 0.80, 0.15], [0.19, 0.01, 0.80]]
        pi = [0.40, 0.30, 0.30]
        B = _gmm_prior([lambda i: i + 1, lambda i: i - 1, lambda i: i - 2], 6.0)
        return A, B, pi

    def init_parameter_state5(self):
        """StructureFind.py:958-1003 (start, downstream, no bias, upstream, end)."""
        A = [[0.00, 1.00, 0.00, 0.00, 0.00], [0.00, 0.50, 0.50, 0.00, 0.00], [0.33, 0.00, 0.34, 0.33, 0.00],
             [0.00, 0.00, 0.00, 0.50, 0.50], [0.50, 0.00, 0.50, 0.00, 0.00]]
        pi = [0.05, 0.3, 0.3, 0.3, 0.05]
        B = _gmm_prior([lambda i: i + 1, lambda i: i, lambda i: i - 1, lambda i: i - 2, lambda i: i - 3], 6.0)
        return A, B, pi

    def init_parameter_state6(self):
        """StructureFind.py:1006-1049 (+ a gap state with variance 1e-4)."""
        A = [[0.00, 1.00, 0.00, 0.00, 0.00, 0.00], [0.00, 0.75, 0.20, 0.00, 0.00, 0.05],
             [0.00, 0.00, 0.60, 0.35, 0.00, 0.05], [0.00, 0.00, 0.00, 0.93, 0.02, 0.05],
             [0.20, 0.60, 0.20, 0.00, 0.00, 0.00], [0.00, 0.22, 0.06, 0.22, 0.00, 0.50]]
        pi = [0.01, 0.29, 0.20, 0.10, 0.05, 0.35]
        B = _gmm_prior([lambda i: i - 3, lambda i: i - 2, lambda i: i - 1, lambda i: i, lambda i: i + 1,
                        lambda i: 0], 4.2)
        B[5][1] = [0.0001, 0.0001, 0.0001]
        return A, B, pi

    def set_model(self, A, B, pi):
        """Install HMM parameters (the output of ghmm's training)."""
        self.model = GaussianMixtureHMM(A, B, pi)
        return self.model

    def modelTrain(self):
        """ghmm Baum-Welch training (StructureFind.py:1091-1110) — not built
        (module docstring).  Uses the installed model."""
        if self.model is None:
            raise NotImplementedError(
                "ghmm Baum-Welch training is not part of this build: install trained parameters with "
                "set_model(A, B, pi) (or the priors, set_model(*self.init_parameter_state3()))")
        return self.model

    # ------------------------------------------------------- preprocessing
    def Data_preprocess(self, Matrix_Dict=None):
        """StructureFind.py:842-915: the per-chromosome matrices from the
        cooler (coolio: balanced with NaN -> 0 for traditional data, raw for
        haplotype data) or given in memory.  Sets Gap_all, DI_dict,
        DI_all_train."""
        if Matrix_Dict is None and getattr(self, "cooler_fil", None):
            return self._data_preprocess_pixels()
        if Matrix_Dict is None:
            Matrix_Dict = getattr(self, "Matrix_Dict", None)
        if Matrix_Dict is None:
            raise ValueError("Data_preprocess needs a cooler file or the per-chromosome matrices")
        window_bin = int(self.window / self.Res)
        width = 7
        Gap_all, DI_dict, DI_all_train = {}, {}, {}
        for chro, matrix in Matrix_Dict.items():
            N = np.shape(matrix)[0]
            tmp = list(self.Get_Gap(matrix))
            if 0 not in tmp:
                tmp.insert(0, 0)
            if N - 1 not in tmp:
                tmp.append(N - 1)
            Gap = np.array(tmp)
            Gap_desity_t = float(Gap.size) / N / 2.0
            DI_sub = self.Get_DI(matrix, Gap, np.ones(N, dtype=np.int64) * window_bin)
            Gap_all[chro] = Gap
            DI_dict[chro] = DI_sub
            DI_all_train[chro] = self.train_segments(Gap, self.Gap_Filter(Gap, matrix), DI_sub, width,
                                                     Gap_desity_t)
        self.DI_all_train, self.DI_dict, self.Gap_all = DI_all_train, DI_dict, Gap_all
        self.Matrix_Dict, self.chroms = Matrix_Dict, list(Matrix_Dict.keys())

    def _data_preprocess_pixels(self):
        """Data_preprocess from the cooler (StructureFind.py:842-915) on its
        pixel table: per chromosome the gap / DI scans run on a band built on
        the GPU from the pixels and ``bins/weight`` (balanced, NaN -> 0, for
        traditional data :853-854; raw for haplotype data :858-865) -- the
        N x N matrix the reference fetches (5 GB for chr1 at 10 kb) never
        exists; bitwise the dense path's gap and DI (``di_scan_pixels``).
        ``Matrix_Dict`` becomes a lazy {chrom: dense} view for Plot_TAD."""
        from .coolio import Cooler
        with Cooler(self.cooler_fil) as c:
            if self.Allelic is False:
                chroms = list(c.chromnames)
            elif self.Allelic in ("Maternal", "Paternal"):
                chroms = [x for x in c.chromnames if x.startswith(self.Allelic[0])]
            else:
                raise ValueError(f"Unkonwn key word {self.Allelic}, Only Maternal, Paternal, False allowed")
            w = c.weights() if self.Allelic is False else None
            width = 7
            Gap_all, DI_dict, DI_all_train = {}, {}, {}
            for chro in chroms:
                lo, hi = c.extent(chro)
                N = hi - lo
                b1, b2, v = c.pixel_rows(lo, hi)
                keep = b2 < hi
                Gap, DI_sub = self.di_scan_pixels(b1[keep], b2[keep], v[keep], w, lo, N)
                Gap_desity_t = float(Gap.size) / N / 2.0
                Gap_all[chro] = Gap
                DI_dict[chro] = DI_sub
                DI_all_train[chro] = self.train_segments(Gap, self.Gap_Filter(Gap, np.empty((N, 0))), DI_sub, width,
                                                         Gap_desity_t)
        self.DI_all_train, self.DI_dict, self.Gap_all = DI_all_train, DI_dict, Gap_all
        self.Matrix_Dict, self.chroms = _LazyMatrices(self.cooler_fil, chroms, self.Allelic is False), chroms

    @staticmethod
    def train_segments(Gap, Gap_fitered, DI_sub, width, Gap_desity_t):
        """The DI segments between kept gap runs (StructureFind.py:897-907)."""
        Gap = np.asarray(Gap)
        out = {}
        for i in range(1, len(Gap_fitered)):
            a, b = Gap_fitered[i - 1], Gap_fitered[i]
            if b - a <= width:
                continue
            if np.sum((a < Gap) & (Gap < b)) / float(b - a - 1) > Gap_desity_t:
                continue
            out[(a + 1, b)] = DI_sub[a + 1:b]
        return out

    # ------------------------------------------------------------ decoding
    def viterbipath(self, DI_dict):
        """ghmm Viterbi per DI segment (StructureFind.py:1113-1123)."""
        model = self.modelTrain()
        return {d: model.viterbi(list(seq)) for d, seq in DI_dict.items()}

    def BoundaryMask(self, origin_range, mask_str):
        """StructureFind.py:1126-1155: for every (pattern, a, b) and every
        window of raw states equal to the pattern (overlapping, left to right)
        mark position i + a as start / i + b as end ('both' when a == b or
        when the mark meets the other kind)."""
        raw = "".join(origin_range["raw_state"])
        state = origin_range["state"]
        for pat, a, b in mask_str:
            i = raw.find(pat)
            while i != -1:
                if a == b:
                    state[i + a] = "both"
                else:
                    if a >= 0:
                        state[i + a] = "both" if state[i + a] == "end" else "start"
                    if b >= 0:
                        state[i + b] = "both" if state[i + b] == "start" else "end"
                i = raw.find(pat, i + 1)
        return state != "none"

    def BoundaryCall(self, paths_sub, Gap_sub, DI_len_sub):
        """StructureFind.py:1158-1188."""
        origin_range = np.zeros((DI_len_sub,), dtype=STATE_DTYPE)
        origin_range["boundary"] = np.arange(DI_len_sub)
        origin_range["raw_state"] = "5"
        origin_range["state"] = "none"
        for d, (path, rely) in paths_sub.items():
            origin_range["raw_state"][d[0]:d[1]] = [str(int(s))[0] for s in path]
            origin_range["rely"][d[0]:d[1]] = rely
        if self.state_num not in MASK_STR:
            # the reference has no rule for 6 states (its mask_boundary is unbound there)
            raise ValueError("boundary rules exist for state_num 3 and 5 only")
        mask_boundary = self.BoundaryMask(origin_range, MASK_STR[self.state_num])
        boundary_index = origin_range[mask_boundary]
        boundary_index["boundary"] = boundary_index["boundary"] * self.Res
        return boundary_index

    def modelPredict(self):
        """StructureFind.py:1191-1209 (with the installed model; needs
        Data_preprocess to have run)."""
        out = {}
        for chrom in self.DI_all_train.keys():
            paths_sub = self.viterbipath(self.DI_all_train[chrom])
            out[chrom] = self.BoundaryCall(paths_sub=paths_sub, Gap_sub=self.Gap_all[chrom],
                                           DI_len_sub=len(self.DI_dict[chrom]))
        self.boundary_index = out

    # ------------------------------------------------------------- domains
    def Candidate_domains(self):
        """StructureFind.py:1212-1229."""
        cand = {}
        for chrom in self.DI_all_train.keys():
            keys = sorted(self.DI_all_train[chrom].keys())
            c = np.zeros((len(keys),), dtype=[("chr", "<U8"), ("start", np.int64), ("end", np.int64)])
            c["chr"] = chrom
            c["start"] = np.array([k[0] for k in keys], dtype=np.int64) * self.Res
            c["end"] = np.array([k[1] for k in keys], dtype=np.int64) * self.Res
            cand[chrom] = c
        self.candidate_domain = cand

    def BoundaryFilter(self):
        """StructureFind.py:1232-1268: boundaries with >= 3 gap bins in the 7
        bins on one side lose that side's role (both sides: dropped)."""
        width = 7
        out = {}
        for chrom in self.boundary_index.keys():
            G = np.asarray(self.Gap_all[chrom])
            bi = self.boundary_index[chrom]
            for k in range(len(bi["boundary"])):
                bb = bi["boundary"][k] / self.Res
                left = np.sum(((bb - width) <= G) & (G <= bb)) >= (width - 1) / 2.0
                right = np.sum((bb <= G) & (G <= bb + width)) >= (width - 1) / 2.0
                st = bi["state"][k]
                if left and right:
                    bi["state"][k] = "none"
                elif left and st != "end":
                    bi["state"][k] = "start"
                elif left and st == "end":
                    bi["state"][k] = "none"
                elif right and st != "start":
                    bi["state"][k] = "end"
                elif right and st == "start":
                    bi["state"][k] = "none"
            out[chrom] = bi["boundary"][bi["state"] != "none"]
        self.boundary_filtered = out

    def BoundaryToDomain(self):
        """StructureFind.py:1271-1342: consecutive (start|both, end|both)
        boundary pairs inside one candidate domain, without long zero-DI runs,
        with <= 1/3 zero DI, of size in [minTAD, maxTAD]."""
        self.Candidate_domains()
        domains = {}
        for chrom in self.boundary_index.keys():
            bnd = self.boundary_index[chrom]["boundary"]
            st = self.boundary_index[chrom]["state"]
            cs, ce = self.candidate_domain[chrom]["start"], self.candidate_domain[chrom]["end"]
            DI = np.asarray(self.DI_dict[chrom])
            starts, ends = [], []
            for ind in range(len(bnd) - 1):
                b0, b1 = bnd[ind], bnd[ind + 1]
                start_i = np.nonzero((cs <= b0) & (b0 <= ce))[0][0]
                end_i = np.nonzero((cs <= b1) & (b1 <= ce))[0][0]
                if start_i != end_i or st[ind] in ("none", "end") or st[ind + 1] in ("none", "start"):
                    continue
                four = three = two = 0
                for jnd in range(int(b0 / self.Res), int(b1 / self.Res - 3)):
                    if np.sum(DI[jnd:jnd + 4] == 0) == 4:
                        four += 1
                        break
                    elif np.sum(DI[jnd:jnd + 3] == 0) == 3:
                        three += 1
                        break
                    elif np.sum(DI[jnd:jnd + 2] == 0) == 2:
                        two += 1
                if four >= 1 or three >= 2 or two >= 3:
                    continue
                if np.sum(DI[int(b0 / self.Res):int(b1 / self.Res)] == 0) > (b1 - b0) / self.Res * (1.0 / 3.0):
                    continue
                if b1 - b0 < self.minTAD or b1 - b0 > self.maxTAD:
                    continue
                starts.append(b0)
                ends.append(b1)
            d = np.zeros((len(starts),), dtype=[("start", np.int64), ("end", np.int64)])
            d["start"] = np.array(starts, dtype=np.int64)
            d["end"] = np.array(ends, dtype=np.int64)
            domains[chrom] = d
        self.Domain_dict = domains

    def tad_domains(self, Matrix_Dict, minTAD=200000, maxTAD=4000000, state_num=3, window=600000,
                    test_type="ttest", model=None):
        """run_TADs' numeric chain (StructureFind.py:1438-1490, files and plots
        aside): DI scan on the GPU, Viterbi with the given (or installed)
        model, boundary calls, filter, domains.  Returns Domain_dict."""
        self.TAD_parameter_init(minTAD=minTAD, maxTAD=maxTAD, state_num=state_num, window=window,
                                test_type=test_type)
        if model is not None:
            self.model = model
        self.Data_preprocess(Matrix_Dict)
        self.modelPredict()
        self.BoundaryFilter()
        self.BoundaryToDomain()
        return self.Domain_dict


class _LazyMatrices(dict):
    """{chrom: dense matrix} fetched from the cooler on first access (only
    Plot_TAD reads Matrix_Dict after Data_preprocess, StructureFind.py:1354)."""

    def __init__(self, uri, chroms, balance):
        super().__init__()
        self._uri, self._order, self._bal = uri, list(chroms), balance

    def __getitem__(self, chro):
        if not dict.__contains__(self, chro):
            if chro not in self._order:
                raise KeyError(chro)
            from .coolio import Cooler
            with Cooler(self._uri) as c:
                M = c.matrix(balance=self._bal).fetch(chro)
            dict.__setitem__(self, chro, np.nan_to_num(M) if self._bal else M)
        return dict.__getitem__(self, chro)

    def keys(self):
        return list(self._order)

    def __iter__(self):
        return iter(self._order)

    def __len__(self):
        return len(self._order)

    def __contains__(self, chro):
        return chro in self._order

    def items(self):
        return [(k, self[k]) for k in self._order]
