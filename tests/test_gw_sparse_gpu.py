"""Sparse GenomeWideMatrixCorrection (csrc/gw.hip) against the reference's
own output (golden, dense) and the oracle, on pixel tables: T as cooler's
upper-triangle table, H as its nonzero ordered cells (matrixBuilding.py:857-901)."""
import numpy as np
import pytest

from oracle import hichap_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mb():
    from hichap_master_amd import _lib, matrixBuilding
    _lib.require_gpu()
    return matrixBuilding


def _tables(T, H):
    i, j = np.nonzero(np.triu(T))
    tp = (i, j, T[i, j])
    r, c = np.nonzero(H)
    return tp, (r, c, H[r, c])


def _layout(names, sizes):
    n = sum(sizes)
    bins, hbins, s = {}, {}, 0
    for nm, L in zip(names, sizes):
        bins[nm] = (s, s + L - 1)
        hbins["M" + nm] = (s, s + L - 1)
        hbins["P" + nm] = (n + s, n + s + L - 1)
        s += L
    return bins, hbins


def _check_upper(b1, b2, v, dense, rtol):
    N = dense.shape[0]
    assert np.all(b1 <= b2)
    key = b1 * N + b2
    assert np.all(np.diff(key) > 0)  # cooler order, unique
    np.testing.assert_allclose(v, dense[b1, b2], rtol=rtol, atol=0)
    # every nonzero of the dense result's upper triangle is present
    iu, ju = np.nonzero(np.triu(dense))
    assert np.array_equal(np.sort(iu * N + ju), np.sort(key[v != 0]))


def test_matches_reference_golden(mb, golden):
    g = golden("genomewide_3chrom")
    bins, hbins = _layout([str(x) for x in g["names"]], [int(x) for x in g["sizes"]])
    tp, hc = _tables(g["T_M"], g["H_M"])
    b1, b2, v = mb.GenomeWideMatrixCorrectionSparse(bins, hbins, tp, hc)
    _check_upper(b1, b2, v, g["Nor"], 1e-12)


@pytest.mark.parametrize("seed", [1, 2])
def test_matches_oracle_with_orphans_and_diagonal(mb, seed):
    """Random asymmetric H with cells whose transposed partner is missing (the
    sum form keeps S_ij alone), diagonal cells, empty rows and a SNP-poor
    stretch; T with gaps."""
    rng = np.random.default_rng(seed)
    sizes = [70, 45, 90]
    n = sum(sizes)
    T = np.triu(rng.poisson(2.0, size=(n, n)) * (rng.random((n, n)) < 0.5))
    T = T + np.triu(T, 1).T
    T[5, :] = T[:, 5] = 0
    H = rng.poisson(0.8, size=(2 * n, 2 * n)) * (rng.random((2 * n, 2 * n)) < 0.3)
    H[10, :] = 0
    H[:, 33] = 0
    bins, hbins = _layout(["1", "2", "X"], sizes)
    tp, hc = _tables(T, H)
    b1, b2, v = mb.GenomeWideMatrixCorrectionSparse(bins, hbins, tp, hc)
    ref = hichap_ref.genome_wide_correction(bins, hbins, T, H)
    _check_upper(b1, b2, v, ref, 1e-12)
    dense = mb.GenomeWideMatrixCorrection(bins, hbins, T, H)
    _check_upper(b1, b2, v, dense, 1e-12)


def test_huge_t_counts_unpacked_path(mb):
    """T counts near 2^32 (count total > 2^40): the packed one-atomic column
    statistics cannot hold the sums, so hh_gw_create reruns them unpacked;
    the result still equals the oracle and the dense path."""
    rng = np.random.default_rng(5)
    sizes = [60, 40]
    n = sum(sizes)
    T = np.triu(rng.poisson(2.0, size=(n, n)) * (rng.random((n, n)) < 0.5)).astype(np.int64)
    T = np.where(T > 0, 3_000_000_000 + T, 0)
    T = T + np.triu(T, 1).T
    assert T.max() < 2**32 and np.triu(T).sum() > 2**40
    H = rng.poisson(0.8, size=(2 * n, 2 * n)) * (rng.random((2 * n, 2 * n)) < 0.3)
    bins, hbins = _layout(["1", "2"], sizes)
    tp, hc = _tables(T, H)
    b1, b2, v = mb.GenomeWideMatrixCorrectionSparse(bins, hbins, tp, hc)
    ref = hichap_ref.genome_wide_correction(bins, hbins, T, H)
    _check_upper(b1, b2, v, ref, 1e-12)


def test_device_tables_and_errors(mb):
    import torch
    from hichap_master_amd._lib import HipLibraryError
    rng = np.random.default_rng(8)
    sizes = [60, 40]
    n = sum(sizes)
    T = np.triu(rng.poisson(3.0, size=(n, n)))
    T = T + np.triu(T, 1).T
    H = rng.poisson(0.6, size=(2 * n, 2 * n))
    bins, hbins = _layout(["1", "2"], sizes)
    tp, hc = _tables(T, H)
    host = mb.GenomeWideMatrixCorrectionSparse(bins, hbins, tp, hc)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).cuda()
    dev = mb.GenomeWideMatrixCorrectionSparse(bins, hbins, [t(x) for x in tp], [t(x) for x in hc],
                                              device_result=True)
    np.testing.assert_array_equal(dev[0].cpu().numpy(), host[0])
    np.testing.assert_array_equal(dev[1].cpu().numpy(), host[1])
    np.testing.assert_array_equal(dev[2].cpu().numpy(), host[2])
    r, c, v = hc
    with pytest.raises(HipLibraryError, match="sorted"):
        mb.GenomeWideMatrixCorrectionSparse(bins, hbins, tp, (r[::-1], c[::-1], v[::-1]))
    with pytest.raises(HipLibraryError, match="upper"):
        mb.GenomeWideMatrixCorrectionSparse(bins, hbins, (tp[1], tp[0], tp[2]), hc)
    bad = dict(hbins)
    bad["P1"] = (0, 59)
    with pytest.raises(ValueError):
        mb.GenomeWideMatrixCorrectionSparse(bins, bad, tp, hc)


def test_device_tables_validated_by_statistics_kernels(mb):
    """int32 device tables are validated inside the statistics kernels (no
    separate check pass): every error code, in either table, is reported with
    the same message and entry as the host tables' separate check, including
    errors at a chunk's first lane and the first entry."""
    import torch
    from hichap_master_amd._lib import HipLibraryError
    rng = np.random.default_rng(21)
    sizes = [900, 700]
    n = sum(sizes)
    T = np.triu(rng.poisson(0.4, size=(n, n)))
    H = rng.poisson(0.25, size=(2 * n, 2 * n))
    bins, hbins = _layout(["1", "2"], sizes)
    tp, hc = _tables(T, H)
    assert tp[0].size > 40000 and hc[0].size > 100000  # several chunks per block
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).cuda()

    def msg(tabs_t, tabs_h, dev):
        conv = (lambda x: [t(a) for a in x]) if dev else (lambda x: [np.asarray(a, dtype=np.int64) for a in x])
        with pytest.raises(HipLibraryError) as e:
            mb.GenomeWideMatrixCorrectionSparse(bins, hbins, conv(tabs_t), conv(tabs_h))
        return str(e.value)

    cases = []
    for which, (r, c, v), nb in (("T", tp, n), ("H", hc, 2 * n)):
        m = r.size
        for at in (0, 2048, 2047 + 64, m // 2 + 1, m - 1):
            for kind in ("range", "order", "dup", "neg") + (("upper",) if which == "T" else ()):
                rr, cc, vv = (np.array(x, dtype=np.int64) for x in (r, c, v))
                if kind == "range":
                    cc[at] = nb
                elif kind == "neg":
                    vv[at] = -3
                elif kind == "upper":
                    rr[at], cc[at] = cc[at] + 1, rr[at]
                elif at > 0:
                    rr[at], cc[at] = rr[at - 1], cc[at - 1] - (kind == "order")
                else:
                    continue
                cases.append((which, (rr, cc, vv)))
    for which, bad in cases:
        tt, hh = (bad, hc) if which == "T" else (tp, bad)
        m_host, m_dev = msg(tt, hh, False), msg(tt, hh, True)
        # the same text after the entry point's name (hh_gw_create vs hh_gw_create_device)
        assert m_host.split(": ", 1)[1] == m_dev.split(": ", 1)[1], (which, m_host, m_dev)


def test_default_wholeres_matches_dense(mb):
    """500 kb diploid hg19 (2n = 12 174): sparse == oracle (dense)."""
    from tests.test_fullsize_gpu import _diploid_inputs
    bins, hap, T, H = _diploid_inputs(500000)
    tp, hc = _tables(T, H)
    b1, b2, v = mb.GenomeWideMatrixCorrectionSparse(bins, hap, tp, hc)
    ref = hichap_ref.genome_wide_correction(bins, hap, T, H)
    np.testing.assert_allclose(v, ref[b1, b2], rtol=1e-11)
    assert b1.size == np.count_nonzero(np.triu(ref))


def _gw_10kb(t_target, h_target):
    """The bench's 10 kb diploid layout (hg19, 2n = 607 282 bins) with
    synthetic T (upper table) and imputed H (ordered cells) in HBM
    (bench.py --config gw at a chosen depth)."""
    from hichap_master_amd import ice, synth
    names = synth.HG19_ORDER
    nb = synth.genome_bins(10000)
    n = int(np.sum(nb))
    At, tdt = synth.calibrate(nb, t_target, 0.2)
    Ah, tdh = synth.calibrate(nb + nb, h_target / 2.0, 0.2)
    T = ice.SynthPixels(nb, ordered=False, A=At, trans_density=tdt, comp_block=200, ignore_diags=0, seed=20201021)
    H = ice.SynthPixels(nb + nb, ordered=True, A=Ah, trans_density=tdh, comp_block=200, ignore_diags=0,
                        seed=20201022)
    off = np.concatenate([[0], np.cumsum(nb)])
    bins = {c: (int(off[k]), int(off[k + 1]) - 1) for k, c in enumerate(names)}
    hap = {}
    for c in names:
        hap["M" + c] = bins[c]
        hap["P" + c] = (n + bins[c][0], n + bins[c][1])
    return bins, hap, T, H, 2 * n


def _host(a):
    import ctypes as C
    import torch
    from hichap_master_amd._lib import call
    t = torch.empty(a.numel(), dtype=torch.int32, device="cuda")
    if a.numel():
        call("hh_device_copy", C.c_void_p(t.data_ptr()), C.c_void_p(a.data_ptr()), 4 * a.numel(), None)
    call("hh_synchronize", None)
    return t.cpu().numpy()


def test_10kb_diploid_layout_matches_sparse_oracle(mb):
    """a4 at its real layout (10 kb diploid, 607 282 bins: every chromosome
    block, the 2n-bin M / P halves, Sort_Chromosomes order) at reduced depth
    (~2e8 T pixels + ~2e8 H cells): the GPU's corrected upper table equals
    the pixel-table oracle (same cells, values to 1e-11)."""
    bins, hap, T, H, N2 = _gw_10kb(2e8, 2e8)
    try:
        assert T.nnz > 1e8 and H.nnz > 1e8
        b1, b2, v = (x.cpu().numpy() for x in
                     mb.GenomeWideMatrixCorrectionSparse(bins, hap, (T.bin1, T.bin2, T.count),
                                                         (H.bin1, H.bin2, H.count), device_result=True))
        tp = tuple(_host(x) for x in (T.bin1, T.bin2, T.count))
        hc = tuple(_host(x) for x in (H.bin1, H.bin2, H.count))
    finally:
        T.close()
        H.close()
    r1, r2, rv = hichap_ref.genome_wide_correction_sparse(bins, hap, tp, hc)
    np.testing.assert_array_equal(b1, r1)
    np.testing.assert_array_equal(b2, r2)
    np.testing.assert_allclose(v, rv, rtol=1e-11, atol=0)


def test_bench_size_invariants(mb):
    """bench.py --config gw's size (1.5e9 T pixels + 1.5e9 H cells): the
    corrected table is sorted and unique upper-triangle (cooler order), and
    the mean rescale's invariant holds, sum(Nor) over the full symmetric
    matrix == sum(H) (matrixBuilding.py:897-899), to 1e-9."""
    import torch
    bins, hap, T, H, N2 = _gw_10kb(1.5e9, 1.5e9)
    try:
        b1, b2, v = mb.GenomeWideMatrixCorrectionSparse(bins, hap, (T.bin1, T.bin2, T.count),
                                                        (H.bin1, H.bin2, H.count), device_result=True)
        import ctypes as C
        from hichap_master_amd._lib import call
        hcnt = torch.empty(H.count.numel(), dtype=torch.int32, device="cuda")
        call("hh_device_copy", C.c_void_p(hcnt.data_ptr()), C.c_void_p(H.count.data_ptr()), 4 * H.count.numel(), None)
        call("hh_synchronize", None)
        hsum = float(hcnt.to(torch.int64).sum().item())
        del hcnt
    finally:
        T.close()
        H.close()
    assert b1.numel() > 1e9
    assert bool((b1 <= b2).all())
    key = b1.to(torch.int64) * N2 + b2.to(torch.int64)
    assert bool((key[1:] > key[:-1]).all())
    del key
    tot = float((torch.where(b1 == b2, 1.0, 2.0).to(torch.float64) * v).sum().item())
    assert abs(tot - hsum) <= 1e-9 * hsum, (tot, hsum)


def test_large_h_counts_index_keys(mb):
    """An H count >= 2^24 does not fit the packed (col | row | count) column
    keys: the column lists fall back to index keys + k_gw_pack; same result
    as the oracle and the dense path."""
    rng = np.random.default_rng(11)
    sizes = [50, 35]
    n = sum(sizes)
    T = np.triu(rng.poisson(2.0, size=(n, n)) * (rng.random((n, n)) < 0.5))
    T = T + np.triu(T, 1).T
    H = (rng.poisson(0.8, size=(2 * n, 2 * n)) * (rng.random((2 * n, 2 * n)) < 0.3)).astype(np.int64)
    H[3, 100] = 2**24 + 5
    H[120, 7] = 2**31
    bins, hbins = _layout(["1", "2"], sizes)
    tp, hc = _tables(T, H)
    b1, b2, v = mb.GenomeWideMatrixCorrectionSparse(bins, hbins, tp, hc)
    ref = hichap_ref.genome_wide_correction(bins, hbins, T, H)
    _check_upper(b1, b2, v, ref, 1e-12)


def test_cpp_alpha_is_numpy_alpha(mb, golden):
    """The alpha step computed in C++ while the column lists build
    (hh_gw_alpha) gives the NumPy expressions' bits: the corrected tables are
    identical, on the reference golden, on random layouts with gaps and on
    the 10 kb diploid layout at reduced depth; a chromosome without non-gap
    bins takes NumPy's path and raises the same error."""
    g = golden("genomewide_3chrom")
    bins, hbins = _layout([str(x) for x in g["names"]], [int(x) for x in g["sizes"]])
    tp, hc = _tables(g["T_M"], g["H_M"])
    a = mb.GenomeWideMatrixCorrectionSparse(bins, hbins, tp, hc)
    b = mb.GenomeWideMatrixCorrectionSparse(bins, hbins, tp, hc, numpy_alpha=True)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    rng = np.random.default_rng(3)
    sizes = [120, 7, 64, 200]
    n = sum(sizes)
    T = np.triu(rng.poisson(1.0, size=(n, n)) * (rng.random((n, n)) < 0.3))
    T[:, 130:140] = 0  # gap rows / columns
    T[130:140, :] = 0
    H = rng.poisson(0.7, size=(2 * n, 2 * n)) * (rng.random((2 * n, 2 * n)) < 0.2)
    bins, hbins = _layout(["1", "2", "3", "X"], sizes)
    tp, hc = _tables(T, H)
    a = mb.GenomeWideMatrixCorrectionSparse(bins, hbins, tp, hc)
    b = mb.GenomeWideMatrixCorrectionSparse(bins, hbins, tp, hc, numpy_alpha=True)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    T2 = T.copy()
    T2[120:127, :] = 0  # chromosome "2": every bin a gap -> np.max of an empty array
    T2[:, 120:127] = 0
    tp2, _ = _tables(T2, H)
    for na in (False, True):
        with pytest.raises(ValueError):
            mb.GenomeWideMatrixCorrectionSparse(bins, hbins, tp2, hc, numpy_alpha=na)
    bins, hap, T, H, N2 = _gw_10kb(2e8, 2e8)  # (at 5e7 some chromosome has no non-gap bin: both paths raise)
    try:
        a = [x.cpu().numpy() for x in mb.GenomeWideMatrixCorrectionSparse(
            bins, hap, (T.bin1, T.bin2, T.count), (H.bin1, H.bin2, H.count), device_result=True)]
        b = [x.cpu().numpy() for x in mb.GenomeWideMatrixCorrectionSparse(
            bins, hap, (T.bin1, T.bin2, T.count), (H.bin1, H.bin2, H.count), device_result=True,
            numpy_alpha=True)]
    finally:
        T.close()
        H.close()
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
