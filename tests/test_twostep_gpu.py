"""HiCHap two-step / genome-wide correction on the GPU vs the reference's own
outputs (golden vectors) and vs the oracle at larger sizes."""
import numpy as np
import pytest

from hichap_master_amd import synth
from oracle import hichap_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mb():
    from hichap_master_amd import _lib, matrixBuilding
    _lib.require_gpu()
    return matrixBuilding


@pytest.mark.parametrize("name", ["twostep_gaps_n96", "twostep_gaps_n160", "twostep_nogapM_n80"])
def test_twostep_matches_reference_golden(mb, golden, name):
    g = golden(name)
    nmm, npm, gm, gp = mb.TwoStepCorrection(g["TM"], g["MM"], g["PM"])
    np.testing.assert_array_equal(gm, g["Gap_M"])
    np.testing.assert_array_equal(gp, g["Gap_P"])
    np.testing.assert_allclose(nmm, g["Nor_MM"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(npm, g["Nor_PM"], rtol=1e-12, atol=0)


@pytest.mark.parametrize("name", ["twostep_gaps_n96", "twostep_gaps_n160", "twostep_nogapM_n80"])
def test_twostep_golden_through_device_batch(mb, golden, name):
    """The reference's own outputs through the path the twostep benches time:
    device tensors into TwoStepCorrection (hh_twostep -> the one-chromosome
    hh_twostep_batch) and into IntraChromMatrixCorrection with shared launches
    (n_streams 0) and with chains on streams; twostep_nogapM_n80 is the SUM
    branch of Trans2symmetry (matrixBuilding.py:948-952)."""
    import torch
    g = golden(name)
    dev = [torch.from_numpy(np.ascontiguousarray(g[k], dtype=np.int64)).cuda() for k in ("TM", "MM", "PM")]
    nmm, npm, gm, gp = mb.TwoStepCorrection(*dev)
    np.testing.assert_array_equal(gm, g["Gap_M"])
    np.testing.assert_array_equal(gp, g["Gap_P"])
    np.testing.assert_allclose(nmm.cpu().numpy(), g["Nor_MM"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(npm.cpu().numpy(), g["Nor_PM"], rtol=1e-12, atol=0)
    for ns in (0, 2):
        nor, gaps = mb.IntraChromMatrixCorrection({"7": dev[0]}, {"M7": dev[1], "P7": dev[2]}, n_streams=ns)
        np.testing.assert_array_equal(gaps["M7"], g["Gap_M"])
        np.testing.assert_array_equal(gaps["P7"], g["Gap_P"])
        np.testing.assert_allclose(nor["M7"].cpu().numpy(), g["Nor_MM"], rtol=1e-12, atol=0)
        np.testing.assert_allclose(nor["P7"].cpu().numpy(), g["Nor_PM"], rtol=1e-12, atol=0)
    # the three goldens as one genome-wide batch (shared launches across
    # chromosomes of different sizes and branches)
    names = ["twostep_gaps_n96", "twostep_gaps_n160", "twostep_nogapM_n80"]
    gs = [golden(nm) for nm in names]
    tra = {str(i): torch.from_numpy(np.ascontiguousarray(x["TM"], dtype=np.int64)).cuda() for i, x in enumerate(gs)}
    hap = {}
    for i, x in enumerate(gs):
        hap["M%d" % i] = torch.from_numpy(np.ascontiguousarray(x["MM"], dtype=np.int64)).cuda()
        hap["P%d" % i] = torch.from_numpy(np.ascontiguousarray(x["PM"], dtype=np.int64)).cuda()
    nor, gaps = mb.IntraChromMatrixCorrection(tra, hap, n_streams=0)
    for i, x in enumerate(gs):
        np.testing.assert_array_equal(gaps["M%d" % i], x["Gap_M"])
        np.testing.assert_array_equal(gaps["P%d" % i], x["Gap_P"])
        np.testing.assert_allclose(nor["M%d" % i].cpu().numpy(), x["Nor_MM"], rtol=1e-12, atol=0)
        np.testing.assert_allclose(nor["P%d" % i].cpu().numpy(), x["Nor_PM"], rtol=1e-12, atol=0)


def test_genomewide_matches_reference_golden(mb, golden):
    g = golden("genomewide_3chrom")
    names = [str(x) for x in g["names"]]
    sizes = [int(x) for x in g["sizes"]]
    n = sum(sizes)
    bins, hbins, s = {}, {}, 0
    for nm, L in zip(names, sizes):
        bins[nm] = (s, s + L - 1)
        hbins["M" + nm] = (s, s + L - 1)
        hbins["P" + nm] = (n + s, n + s + L - 1)
        s += L
    out = mb.GenomeWideMatrixCorrection(bins, hbins, g["T_M"], g["H_M"])
    np.testing.assert_allclose(out, g["Nor"], rtol=1e-12, atol=0)


@pytest.mark.parametrize("N,drop", [(1000, 40), (777, 0), (130, 5)])
def test_twostep_vs_oracle_sizes(mb, N, drop):
    rng = np.random.default_rng(N)
    TM = synth.dense_chrom(N, rng, A=60.0)
    MM, PM = synth.haplotype_pair(TM, rng, drop_rows=drop)
    got = mb.TwoStepCorrection(TM, MM, PM)
    ref = hichap_ref.two_step_correction(TM, MM, PM)
    np.testing.assert_array_equal(got[2], ref[2])
    np.testing.assert_array_equal(got[3], ref[3])
    for a, b in zip(got[:2], ref[:2]):
        np.testing.assert_allclose(a, b, rtol=1e-11, atol=0)
        # size-independent invariants: symmetric, sum preserved (mean rescale)
        np.testing.assert_array_equal(a, a.T)
    np.testing.assert_allclose(got[0].sum(), MM.sum(), rtol=1e-9)


def test_intra_chrom_dict_api(mb):
    rng = np.random.default_rng(5)
    tra, hap = {}, {}
    for c, N in (("1", 90), ("X", 70)):
        TM = synth.dense_chrom(N, rng, A=50.0)
        tra[c] = TM
        hap["M" + c], hap["P" + c] = synth.haplotype_pair(TM, rng, drop_rows=3)
    nor, gaps = mb.IntraChromMatrixCorrection(tra, hap)
    assert set(nor) == {"M1", "P1", "MX", "PX"}
    ref = hichap_ref.two_step_correction(tra["X"], hap["MX"], hap["PX"])
    np.testing.assert_allclose(nor["PX"], ref[1], rtol=1e-11)
    np.testing.assert_array_equal(gaps["MX"], ref[2])


@pytest.mark.parametrize("N,drop", [(6232, 120), (4813, 60)])
def test_twostep_real_sizes_vs_oracle(mb, N, drop):
    """TwoStepCorrection at HiCHap's own sizes: chr1 at the default localRes
    40 kb (N = 249 250 621 // 40 000 + 1 = 6 232) and chr21 at 10 kb
    (N = 48 129 895 // 10 000 + 1 = 4 813), against the oracle."""
    rng = np.random.default_rng(N)
    TM = synth.dense_chrom(N, rng, A=60.0)
    MM, PM = synth.haplotype_pair(TM, rng, drop_rows=drop)
    got = mb.TwoStepCorrection(TM, MM, PM)
    ref = hichap_ref.two_step_correction(TM, MM, PM)
    np.testing.assert_array_equal(got[2], ref[2])
    np.testing.assert_array_equal(got[3], ref[3])
    for a, b in zip(got[:2], ref[:2]):
        np.testing.assert_allclose(a, b, rtol=1e-11, atol=0)
    np.testing.assert_allclose(got[1].sum(), PM.sum(), rtol=1e-9)


def test_twostep_from_cells_and_device(mb):
    """The PCIe-free forms: dense matrices built on the GPU from the tables
    (T upper pixels, MM / PM ordered cells, global ids) and corrected there,
    returned as upper tables or device tensors -- bitwise the host-array
    TwoStepCorrection (same kernels on the same matrices)."""
    import torch
    N, off = 1500, 1000
    rng = np.random.default_rng(77)
    TM = synth.dense_chrom(N, rng, A=60.0)
    MM, PM = synth.haplotype_pair(TM, rng, drop_rows=30)
    want = mb.TwoStepCorrection(TM, MM, PM)
    i, j = np.nonzero(np.triu(TM))
    tp = (i + off, j + off, TM[i, j])
    cells = []
    for X in (MM, PM):
        r, c = np.nonzero(X)
        cells.append((r + off, c + off, X[r, c]))
    um, up, gm, gp = mb.TwoStepCorrectionPixels(N, tp, cells[0], cells[1], offset=off)
    np.testing.assert_array_equal(gm, want[2])
    np.testing.assert_array_equal(gp, want[3])
    for (b1, b2, v), D in ((um, want[0]), (up, want[1])):
        r, c = np.nonzero(np.triu(D))
        np.testing.assert_array_equal(b1, r + off)
        np.testing.assert_array_equal(b2, c + off)
        np.testing.assert_array_equal(v, D[r, c])
    dev = [torch.from_numpy(X).cuda() for X in (TM, MM, PM)]
    nm, npm, gm2, gp2 = mb.TwoStepCorrection(*dev)
    np.testing.assert_array_equal(nm.cpu().numpy(), want[0])
    np.testing.assert_array_equal(npm.cpu().numpy(), want[1])
    np.testing.assert_array_equal(gm2, want[2])
    # device cells too
    tcells = [torch.from_numpy(np.asarray(x, np.int64)).cuda() for x in tp]
    D = mb.dense_from_cells_device(tcells, N, off, symmetric=True)
    np.testing.assert_array_equal(D.cpu().numpy(), TM)
    from hichap_master_amd._lib import HipLibraryError
    with pytest.raises(HipLibraryError, match="outside"):
        mb.dense_from_cells_device((np.array([off + N]), np.array([off]), np.array([1])), N, off)


def test_dense_from_cells_repeated_cells_add_up(mb):
    """Repeated (row, col) cells add up, as the reference's per-line
    `Matrix[bin1][bin2] += 1` does (matrixBuilding.py:1291-1301): ordered and
    symmetric tables, diagonal cells counted once, run-to-run identical."""
    rng = np.random.default_rng(91)
    N, off = 300, 50
    r = rng.integers(0, N, 20000)
    c = rng.integers(0, N, 20000)
    v = rng.integers(1, 5, 20000)
    want = np.zeros((N, N), np.int64)
    np.add.at(want, (r, c), v)
    D = mb.dense_from_cells_device((r + off, c + off, v), N, off)
    np.testing.assert_array_equal(D.cpu().numpy(), want)
    a, b = np.minimum(r, c), np.maximum(r, c)
    ws = np.zeros((N, N), np.int64)
    np.add.at(ws, (a, b), v)
    ws = ws + np.triu(ws, 1).T
    for _ in range(2):
        D = mb.dense_from_cells_device((a + off, b + off, v), N, off, symmetric=True)
        np.testing.assert_array_equal(D.cpu().numpy(), ws)


def test_twostep_cpu_torch_tensors_take_the_host_path(mb):
    """CPU torch tensors have data_ptr too: they go the host-array way
    (ADVICE r3), not to the device-tensor form."""
    import torch
    N = 200
    rng = np.random.default_rng(92)
    TM = synth.dense_chrom(N, rng, A=60.0)
    MM, PM = synth.haplotype_pair(TM, rng, drop_rows=5)
    want = mb.TwoStepCorrection(TM, MM, PM)
    got = mb.TwoStepCorrection(*(torch.from_numpy(X) for X in (TM, MM, PM)))
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)
    with pytest.raises(ValueError):
        mb.TwoStepCorrection(torch.from_numpy(TM).cuda(), MM, PM)


def _twostep_with(mb, tune, *mats):
    from hichap_master_amd import _lib
    try:
        for k, v in tune.items():
            _lib.call("hh_tune", k.encode(), int(v))
        return mb.TwoStepCorrection(*mats)
    finally:
        _lib.call("hh_tune", b"symvc_stream", 1)
        _lib.call("hh_tune", b"symvc_out", 1)
        _lib.call("hh_tune", b"symvc_rows", 32)
        _lib.call("hh_tune", b"twostep_devglue", 1)


@pytest.mark.parametrize("case", ["gaps_1000", "nogap_golden", "ragged_777"])
def test_twostep_streaming_passes_match_tile_pairs(mb, golden, case):
    """Passes 1-2 as row streams (k_ts_gemv + the both-gap correction) give
    the tile-pair passes' result up to summation rounding, with the gap and
    the no-gap (sum) forms; the one-LDS-tile pass 3 is bitwise the two-tile
    one; the rows-per-block knob does not change the result beyond rounding;
    the gap / alpha glue on the device gives the host glue's bits."""
    if case == "nogap_golden":
        g = golden("twostep_nogapM_n80")
        mats = (g["TM"], g["MM"], g["PM"])
    else:
        N, drop = (1000, 40) if case == "gaps_1000" else (777, 0)
        rng = np.random.default_rng(N + 7)
        TM = synth.dense_chrom(N, rng, A=60.0)
        mats = (TM,) + tuple(synth.haplotype_pair(TM, rng, drop_rows=drop))
    tiles = _twostep_with(mb, {"symvc_stream": 0, "symvc_out": 0}, *mats)
    stream2 = _twostep_with(mb, {"symvc_stream": 1, "symvc_out": 0}, *mats)
    stream1 = _twostep_with(mb, {"symvc_stream": 1, "symvc_out": 1}, *mats)
    rows16 = _twostep_with(mb, {"symvc_rows": 16}, *mats)
    hostglue = _twostep_with(mb, {"twostep_devglue": 0}, *mats)
    for k in range(4):  # the device glue (gaps, alpha, raw totals) is bitwise the host glue
        np.testing.assert_array_equal(stream1[k], hostglue[k])
    for k in (2, 3):
        np.testing.assert_array_equal(stream1[k], tiles[k])
    for k in (0, 1):
        np.testing.assert_allclose(stream1[k], tiles[k], rtol=1e-13, atol=0)
        np.testing.assert_array_equal(stream1[k], stream2[k])
        np.testing.assert_allclose(rows16[k], stream1[k], rtol=1e-13, atol=0)
        np.testing.assert_array_equal(stream1[k], stream1[k].T)


@pytest.mark.parametrize("devglue", [1, 0])
def test_twostep_all_zero_haplotype_raises(mb, devglue):
    """An all-zero haplotype matrix has no nonzero coverage: NumPy's
    percentile of an empty array raises in the reference (Gap_defined :922);
    both glue paths raise instead of returning garbage."""
    from hichap_master_amd import _lib
    N = 200
    rng = np.random.default_rng(5)
    TM = synth.dense_chrom(N, rng, A=60.0)
    Z = np.zeros_like(TM)
    with pytest.raises(_lib.HipLibraryError, match="percentile of an empty array"):
        _twostep_with(mb, {"twostep_devglue": devglue}, TM, Z, Z)


def test_twostep_devglue_block_select_path_bitwise(mb):
    """N > 16384 (kSelPer * 1024) takes the device glue's second percentile
    path (block_kth + LDS atomics, dense.hip block_percentile); its gaps,
    alpha and outputs are bitwise the host glue's."""
    import torch
    N = 16500
    g = torch.Generator(device="cuda").manual_seed(11)
    i = torch.arange(N, device="cuda", dtype=torch.float64)
    lam = 40.0 / ((i[:, None] - i[None, :]).abs() + 1.0)
    TM = torch.poisson(lam, generator=g).to(torch.int64)
    TM = torch.triu(TM) + torch.triu(TM, 1).T
    MM = torch.poisson(0.4 * lam, generator=g).to(torch.int64)
    PM = torch.poisson(0.4 * lam, generator=g).to(torch.int64)
    del lam
    MM[100:400] = 0  # gap rows: the gap form of Trans2symmetry
    PM[9000:9100] = 0
    torch.cuda.synchronize()
    dev = _twostep_with(mb, {"twostep_devglue": 1}, TM, MM, PM)
    host = _twostep_with(mb, {"twostep_devglue": 0}, TM, MM, PM)
    for a, b in zip(dev, host):
        if hasattr(a, "device"):
            assert torch.equal(torch.as_tensor(a), torch.as_tensor(b))
        else:
            np.testing.assert_array_equal(a, b)
    gm = dev[2].cpu().numpy() if hasattr(dev[2], "cpu") else dev[2]
    assert 300 <= len(gm) < N  # the zeroed rows are gaps, most rows are not



def _per_chrom_host(mb, T, M, P):
    """The per-chromosome hh_twostep chain on host arrays (the device path of
    TwoStepCorrection runs the one-chromosome batch): float64 CPU tensors and
    the gap arrays."""
    import torch
    one = mb.TwoStepCorrection(*(X.cpu().numpy() for X in (T, M, P)))
    return torch.from_numpy(one[0]), torch.from_numpy(one[1]), one[2], one[3]

@pytest.mark.parametrize("n_streams", [0, 1, 4])
def test_intra_chrom_batch_equals_per_chromosome(mb, n_streams):
    """IntraChromMatrixCorrection on device tensors: every chromosome in one
    hh_twostep_batch call (0: shared launches per pass; else the chains on
    several streams, largest first) is bitwise the per-chromosome
    hh_twostep, gaps included; one chromosome with gap rows, one without,
    sizes from 37 to 2 100 bins."""
    import torch
    rng = np.random.default_rng(77)
    tra, hap = {}, {}
    for c, N, drop in (("1", 2100, 40), ("2", 1500, 0), ("3", 37, 0), ("X", 900, 12), ("4", 1200, 25)):
        TM = synth.dense_chrom(N, rng, A=50.0)
        MM, PM = synth.haplotype_pair(TM, rng, drop_rows=drop)
        tra[c] = torch.from_numpy(TM).cuda()
        hap["M" + c], hap["P" + c] = torch.from_numpy(MM).cuda(), torch.from_numpy(PM).cuda()
    nor, gaps = mb.IntraChromMatrixCorrection(tra, hap, n_streams=n_streams)
    assert set(nor) == {h + c for c in tra for h in "MP"}
    for c in tra:
        one = _per_chrom_host(mb, tra[c], hap["M" + c], hap["P" + c])
        assert torch.equal(nor["M" + c].cpu(), one[0]) and torch.equal(nor["P" + c].cpu(), one[1])
        dev = mb.TwoStepCorrection(tra[c], hap["M" + c], hap["P" + c])  # device: the one-chromosome batch
        assert torch.equal(dev[0], nor["M" + c]) and torch.equal(dev[1], nor["P" + c])
        np.testing.assert_array_equal(gaps["M" + c], one[2])
        np.testing.assert_array_equal(gaps["P" + c], one[3])
    ref = hichap_ref.two_step_correction(tra["X"].cpu().numpy(), hap["MX"].cpu().numpy(), hap["PX"].cpu().numpy())
    np.testing.assert_allclose(nor["MX"].cpu().numpy(), ref[0], rtol=1e-11)
    np.testing.assert_array_equal(gaps["PX"], ref[3])


@pytest.mark.parametrize("n_streams", [0, 3])
def test_intra_chrom_batch_memory_budget_bitwise(mb, n_streams):
    """hh_twostep_batch splits the chromosomes into consecutive groups whose
    workspace fits a device-memory budget (the workspace grows
    with the sum over chromosomes); with a budget so small that every
    chromosome is its own group the results are bitwise those of one batch,
    and an error still names the chromosome by its index in the call."""
    import torch
    from hichap_master_amd import _lib
    rng = np.random.default_rng(91)
    tra, hap = {}, {}
    for c, N, drop in (("1", 1700, 30), ("2", 64, 0), ("3", 1100, 0), ("4", 800, 9)):
        TM = synth.dense_chrom(N, rng, A=50.0)
        MM, PM = synth.haplotype_pair(TM, rng, drop_rows=drop)
        tra[c] = torch.from_numpy(TM).cuda()
        hap["M" + c], hap["P" + c] = torch.from_numpy(MM).cuda(), torch.from_numpy(PM).cuda()
    full, gfull = mb.IntraChromMatrixCorrection(tra, hap, n_streams=n_streams)
    for mbytes in (1, 40):
        _lib.call("hh_tune", b"twostep_budget_mb", mbytes)
        try:
            part, gpart = mb.IntraChromMatrixCorrection(tra, hap, n_streams=n_streams)
        finally:
            _lib.call("hh_tune", b"twostep_budget_mb", 0)
        for k in full:
            assert torch.equal(part[k], full[k]), (mbytes, k)
            np.testing.assert_array_equal(gpart[k], gfull[k])
    Z = torch.zeros_like(tra["3"])
    bad = dict(hap, M3=Z, P3=Z)
    _lib.call("hh_tune", b"twostep_budget_mb", 1)
    try:
        with pytest.raises(_lib.HipLibraryError, match=r"percentile of an empty array \(chromosome 2\)"):
            mb.IntraChromMatrixCorrection(tra, bad, n_streams=n_streams)
    finally:
        _lib.call("hh_tune", b"twostep_budget_mb", 0)
    # the library is usable after the failed call (its buffers were not
    # handed back while kernels still wrote them)
    again, _ = mb.IntraChromMatrixCorrection(tra, hap, n_streams=n_streams)
    for k in full:
        assert torch.equal(again[k], full[k])


def test_intra_chrom_batch_error_names_the_chromosome(mb):
    import torch
    from hichap_master_amd import _lib
    rng = np.random.default_rng(3)
    TM = synth.dense_chrom(300, rng, A=60.0)
    MM, PM = synth.haplotype_pair(TM, rng)
    d = lambda X: torch.from_numpy(np.ascontiguousarray(X)).cuda()
    Z = np.zeros_like(TM)
    tra = {"1": d(TM), "2": d(TM)}
    hap = {"M1": d(MM), "P1": d(PM), "M2": d(Z), "P2": d(Z)}
    with pytest.raises(_lib.HipLibraryError, match=r"percentile of an empty array \(chromosome 1\)"):
        mb.IntraChromMatrixCorrection(tra, hap)


def test_intra_chrom_batch_escaped_counts(mb):
    """The shared-launch batch reads 16-bit copies of MM / PM; counts of
    0xFFFF and above (here 65 535, 65 536, 70 000 and 3e9, on and off the
    diagonal, in both triangles) are stored as 0xFFFF and read from the int64
    matrix: still bitwise the per-chromosome result."""
    import torch
    rng = np.random.default_rng(79)
    tra, hap = {}, {}
    for c, N in (("1", 700), ("2", 130), ("3", 64)):
        TM = synth.dense_chrom(N, rng, A=50.0)
        MM, PM = synth.haplotype_pair(TM, rng, drop_rows=5)
        for (i, j), v in (((0, 0), 65535), ((3, 10), 65536), ((10, 3), 70000), ((N - 1, N - 1), 3_000_000_000),
                          ((N // 2, 1), 65535), ((1, N // 2), 123456)):
            MM[i, j] = v
            PM[j, i] = v + 1
            TM[i, j] += 2 * v
            TM[j, i] = TM[i, j]
        tra[c] = torch.from_numpy(TM).cuda()
        hap["M" + c], hap["P" + c] = torch.from_numpy(MM).cuda(), torch.from_numpy(PM).cuda()
    nor, gaps = mb.IntraChromMatrixCorrection(tra, hap, n_streams=0)
    for c in tra:
        one = _per_chrom_host(mb, tra[c], hap["M" + c], hap["P" + c])
        assert torch.equal(nor["M" + c].cpu(), one[0]) and torch.equal(nor["P" + c].cpu(), one[1])
        np.testing.assert_array_equal(gaps["M" + c], one[2])
        np.testing.assert_array_equal(gaps["P" + c], one[3])


def test_intra_chrom_batch_wide_counts_fallback(mb):
    """The shared-launch batch reads 16-bit copies of MM / PM (escapes up to
    32 bits); a chromosome whose counts do not fit (here one cell of 2^33)
    falls back to the int64
    matrix for its own passes: still bitwise the per-chromosome result."""
    import torch
    rng = np.random.default_rng(78)
    tra, hap = {}, {}
    for c, N, big in (("1", 700, True), ("2", 500, False)):
        TM = synth.dense_chrom(N, rng, A=50.0)
        MM, PM = synth.haplotype_pair(TM, rng, drop_rows=5)
        if big:
            MM[3, 10] = 2 ** 33
            TM[3, 10] = TM[10, 3] = 2 ** 34
        tra[c] = torch.from_numpy(TM).cuda()
        hap["M" + c], hap["P" + c] = torch.from_numpy(MM).cuda(), torch.from_numpy(PM).cuda()
    nor, gaps = mb.IntraChromMatrixCorrection(tra, hap, n_streams=0)
    for c in tra:
        one = _per_chrom_host(mb, tra[c], hap["M" + c], hap["P" + c])
        assert torch.equal(nor["M" + c].cpu(), one[0]) and torch.equal(nor["P" + c].cpu(), one[1])
        np.testing.assert_array_equal(gaps["M" + c], one[2])
