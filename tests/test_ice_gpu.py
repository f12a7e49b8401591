"""ICE on the GPU (through the C-ABI) against the CPU oracle."""
import numpy as np
import pytest

from hichap_master_amd import synth
from oracle import ice_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ice():
    from hichap_master_amd import _lib, ice as ice_mod
    _lib.require_gpu()
    return ice_mod


def _case(seed, sizes=(400, 300), A=25.0, trans=0.01, **kw):
    rng = np.random.default_rng(seed)
    return synth.coo_genome(list(sizes), rng, A=A, trans_density=trans, **kw)


def _filtered_upper(b1, b2, c, off, ignore_diags, cis_only):
    chrom = np.repeat(np.arange(len(off) - 1), np.diff(off))
    keep = (c != 0) & (b2 - b1 >= ignore_diags)
    if cis_only:
        keep &= chrom[b1] == chrom[b2]
    o = np.lexsort((b2[keep], b1[keep]))
    return b1[keep][o], b2[keep][o], c[keep][o].astype(np.float64)


@pytest.mark.parametrize("ignore_diags,cis_only", [(1, False), (0, False), (2, True)])
def test_export_roundtrip(ice, ignore_diags, cis_only):
    b1, b2, c, off = _case(1)
    n = int(off[-1])
    m = ice.ContactMatrix.from_pixels(b1, b2, c, n, off, ignore_diags, cis_only)
    e1, e2, ec = m.export_upper()
    f1, f2, fc = _filtered_upper(b1, b2, c, off, ignore_diags, cis_only)
    np.testing.assert_array_equal(e1, f1)
    np.testing.assert_array_equal(e2, f2)
    np.testing.assert_array_equal(ec, fc)
    assert m.info()["nnz_upper"] == f1.size


@pytest.mark.parametrize("seed", [2, 3])
@pytest.mark.parametrize("cis_only", [False, True])
def test_balance_matches_oracle(ice, seed, cis_only):
    b1, b2, c, off = _case(seed, sizes=(500, 350, 200))
    n = int(off[-1])
    w, st = ice.balance(b1, b2, c, n, off, cis_only=cis_only, max_iters=500)
    wr, sr = ice_ref.balance(b1, b2, c, n, off, cis_only=cis_only, max_iters=500)
    np.testing.assert_array_equal(np.isnan(w), np.isnan(wr))
    np.testing.assert_allclose(w, wr, rtol=1e-9, equal_nan=True)
    np.testing.assert_allclose(st["scale"], sr["scale"], rtol=1e-9)
    np.testing.assert_array_equal(st["iters"], sr["iters"])
    assert st["converged"] == sr["converged"]


def test_balance_unconverged_cap(ice):
    b1, b2, c, off = _case(4)
    n = int(off[-1])
    w, st = ice.balance(b1, b2, c, n, off, max_iters=7)
    wr, sr = ice_ref.balance(b1, b2, c, n, off, max_iters=7)
    assert st["iters"] == 7 and not st["converged"]
    np.testing.assert_allclose(st["var"], sr["var"], rtol=1e-9)
    np.testing.assert_allclose(w, wr, rtol=1e-10, equal_nan=True)


def test_large_counts(ice):
    """Counts up to 2^32-1 fit: a chunk's (count, column-offset) bit split adapts."""
    b1, b2, c, off = _case(5, sizes=(300,), A=40.0, trans=0.0)
    c = c.astype(np.int64)
    rng = np.random.default_rng(0)
    big = rng.random(c.size) < 0.05
    c[big] = c[big] * 40000 + rng.integers(0, 70000, size=big.sum())
    c[np.argmax(c)] = 2**32 - 1
    n = int(off[-1])
    m = ice.ContactMatrix.from_pixels(b1, b2, c, n, off)
    _, _, ec = m.export_upper()
    f1, f2, fc = _filtered_upper(b1, b2, c, off, 1, False)
    np.testing.assert_array_equal(ec, fc)
    w, st = ice.balance_matrix(m, ice.IceOptions(max_iters=300))
    wr, sr = ice_ref.balance(b1, b2, c, n, off, max_iters=300)
    np.testing.assert_allclose(w, wr, rtol=1e-9, equal_nan=True)


def test_diag_kept_and_unsorted_input(ice):
    b1, b2, c, off = _case(6, sizes=(250,), trans=0.0)
    perm = np.random.default_rng(1).permutation(b1.size)
    n = int(off[-1])
    w, st = ice.balance(b1[perm], b2[perm], c[perm], n, off, ignore_diags=0, max_iters=400)
    wr, sr = ice_ref.balance(b1, b2, c, n, off, ignore_diags=0, max_iters=400)
    np.testing.assert_allclose(w, wr, rtol=1e-9, equal_nan=True)


def test_empty_chromosome_cis_only(ice):
    b1, b2, c, off = _case(7, sizes=(200, 60, 150), trans=0.0)
    chrom = np.repeat(np.arange(3), np.diff(off))
    keep = chrom[b1] != 1
    n = int(off[-1])
    w, st = ice.balance(b1[keep], b2[keep], c[keep], n, off, cis_only=True, max_iters=400)
    wr, sr = ice_ref.balance(b1[keep], b2[keep], c[keep], n, off, cis_only=True, max_iters=400)
    assert np.isnan(w[200:260]).all()
    np.testing.assert_allclose(w, wr, rtol=1e-9, equal_nan=True)
    assert np.isnan(st["scale"][1]) and np.isnan(sr["scale"][1])


def test_cis_only_empty_group_between_active_ones(ice):
    """--cis-only with a chromosome whose bins all fail the filters between
    two active ones: cooler gives it NaN weights at its first iteration; that
    NaN must not reach the neighbours' rows through the dense bands' zero
    slots across the chromosome boundaries (it once did: 0 * NaN)."""
    b1, b2, c, off = _case(9, sizes=(500, 300, 400), A=40.0, trans=0.0)
    chrom = np.repeat(np.arange(3), np.diff(off))
    mid = chrom[b1] == 1
    keep = ~mid | (np.arange(b1.size) % 97 == 0)  # a few pixels: every bin < min_nnz
    b1, b2, c = b1[keep], b2[keep], c[keep]
    n = int(off[-1])
    w, st = ice.balance(b1, b2, c, n, off, cis_only=True, max_iters=300)
    wr, sr = ice_ref.balance(b1, b2, c, n, off, cis_only=True, max_iters=300)
    assert np.isnan(w[500:800]).all() and np.isfinite(w[:500]).any() and np.isfinite(w[800:]).any()
    np.testing.assert_array_equal(np.isnan(w), np.isnan(wr))
    np.testing.assert_allclose(w, wr, rtol=1e-9, equal_nan=True)
    np.testing.assert_array_equal(st["iters"], sr["iters"])


def test_invalid_counts_rejected(ice):
    from hichap_master_amd._lib import HipLibraryError
    with pytest.raises(HipLibraryError):
        ice.ContactMatrix.from_pixels([0, 1], [5, 6], [1.5, 2.0], 10, [0, 10])
    with pytest.raises(HipLibraryError):
        ice.ContactMatrix.from_pixels([0, 1], [5, 60], [1, 2], 10, [0, 10])


def _sharded_weights(ice, b1, b2, c, off, rr, max_iters=300):
    """Row shards on one GPU with a manual marginal gather (the sharded
    driver's exchange, without a process group; the column side of
    upper-triangle tiles through one thread per shard)."""
    from tests.shard_exchange import balance_states
    n = int(off[-1])
    opts = ice.IceOptions(max_iters=max_iters)
    W = len(rr) - 1
    shards = [ice.ContactMatrix.from_pixels(b1, b2, c, n, off, row_range=(rr[k], rr[k + 1])) for k in range(W)]
    states = [ice.IceState(m, opts) for m in shards]
    try:
        res = balance_states(states, rr, max_iters)
    finally:
        for st_ in states:
            st_.close()
        for m in shards:
            m.close()
    for w, _ in res[1:]:
        np.testing.assert_array_equal(w, res[0][0])
    return res[0]


def test_sharded_equals_full_bitwise(ice):
    """Two row shards on one GPU with a manual gather == the one-shard run."""
    from hichap_master_amd import dist
    b1, b2, c, off = _case(8, sizes=(500, 400))
    n = int(off[-1])
    w_full, st_full = ice.balance(b1, b2, c, n, off, max_iters=300)
    rr = dist.partition_rows(np.bincount(b1, minlength=n) + np.bincount(b2, minlength=n), 2)
    w0, s0 = _sharded_weights(ice, b1, b2, c, off, rr)
    np.testing.assert_array_equal(w0, w_full)
    assert s0["iters"] == st_full["iters"]


def test_synthetic_generator_matches_oracle(ice):
    sizes = [700, 500, 300]
    kw = dict(A=40.0, trans_density=0.002, comp_block=50, seed=11)
    m = ice.ContactMatrix.synthetic(sizes, **kw)
    inf = m.info()
    b1, b2, c = m.export_upper()
    assert inf["nnz_upper"] == b1.size
    assert (b2 - b1 >= 1).all()
    # symmetric storage: every pixel appears in both rows -> entries = 2 * pixels
    assert inf["n_entries"] == 2 * b1.size
    assert inf["n_slots"] + inf["n_slots_narrow"] + inf["n_band"] >= inf["n_entries"]
    assert inf["n_slots"] % 4 == 0 and inf["n_slots_narrow"] % 8 == 0
    rows = inf["row_hi"] - inf["row_lo"]
    band_bytes = (2 * inf["band_w"] + 16 if inf["band_w"] else 0) * rows
    if inf["band_w4"] > inf["band_w"]:  # 4-bit band: two segments of (W4 - W8) / 2 + 16 bytes
        band_bytes += (inf["band_w4"] - inf["band_w"] + 32) * rows
    assert inf["payload_bytes"] == 4 * inf["n_slots"] + 2 * inf["n_slots_narrow"] + band_bytes
    assert inf["n_slots_narrow"] > 0  # low counts are stored as uint16
    # shards see the same matrix
    rc, ru = ice.synth_row_counts(sizes, **kw)
    assert ru.sum() == b1.size
    half = ice.ContactMatrix.synthetic(sizes, row_range=(0, 1024), **kw)
    h1, h2, hc = half.export_upper()
    sel = b1 < 1024
    np.testing.assert_array_equal(h1, b1[sel]); np.testing.assert_array_equal(h2, b2[sel])
    np.testing.assert_array_equal(hc, c[sel])
    off = m.chrom_offsets
    w, st = ice.balance_matrix(m, ice.IceOptions(max_iters=400))
    wr, sr = ice_ref.balance(b1, b2, c, int(off[-1]), off, max_iters=400)
    np.testing.assert_allclose(w, wr, rtol=1e-9, equal_nan=True)
    assert st["iters"] == sr["iters"]


def test_synth_dense_block_matches_sparse_generator(ice):
    """hh_synth_dense (C5 bench inputs) is the cis block of the same genome."""
    import torch
    sizes = [300, 260]
    kw = dict(A=40.0, trans_density=0.0, comp_block=50, ignore_diags=0, cis_only=True, seed=7)
    m = ice.ContactMatrix.synthetic(sizes, **kw)
    b1, b2, c = m.export_upper()
    off = np.concatenate([[0], np.cumsum(sizes)])
    for k, n in enumerate(sizes):
        buf = torch.zeros((n, n), dtype=torch.float64, device="cuda")
        ice.synth_dense(sizes, k, buf.data_ptr(), **kw)
        D = buf.cpu().numpy()
        np.testing.assert_array_equal(D, D.T)
        want = np.zeros((n, n))
        sel = (b1 >= off[k]) & (b1 < off[k + 1])
        want[b1[sel] - off[k], b2[sel] - off[k]] = c[sel]
        np.testing.assert_array_equal(np.triu(D), want)


def test_balance_sharded_rccl_world1(ice):
    """dist.balance_sharded over a real RCCL process group (world 1): the
    all-gather path through torch.distributed "nccl" gives the full result."""
    import socket
    import torch
    import torch.distributed as tdist
    from hichap_master_amd import dist
    b1, b2, c, off = _case(12, sizes=(600, 350))
    n = int(off[-1])
    w_full, st_full = ice.balance(b1, b2, c, n, off, max_iters=300)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    tdist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                             device_id=torch.device("cuda", 0))
    try:
        rr = np.array([0, n], dtype=np.int64)
        m = ice.ContactMatrix.from_pixels(b1, b2, c, n, off, row_range=(0, n))
        st = ice.IceState(m, ice.IceOptions(max_iters=300))
        ex = dist.Exchange(rr, torch.device("cuda", 0))
        assert ex.fused
        w, s_ = dist.balance_sharded(st, ex, max_iters=300)
    finally:
        tdist.destroy_process_group()
    np.testing.assert_array_equal(w, w_full)
    assert s_["iters"] == st_full["iters"]


@pytest.mark.parametrize("band_w,band4", [(0, 1), (16, 1), (64, 1), (-1, 0), (-1, 1)])
def test_dense_band_widths(ice, band_w, band4):
    """The dense diagonal bands (uint8 of any width or none; the 4-bit band
    beyond it, on or off) hold exactly the pixels they claim: export round
    trip (counts > 255 near the diagonal and > 15 in the 4-bit range go to
    the tiles), and weights equal the oracle's."""
    from hichap_master_amd import _lib
    b1, b2, c, off = _case(31, sizes=(1400, 900), A=60.0, trans=0.02)
    c = c.copy()
    c[::97] = 300   # counts > 255 near the diagonal go to the tiles
    c[5::89] = 16   # ... and counts > 15 in the 4-bit range
    n = int(off[-1])
    _lib.call("hh_tune", b"band_w", band_w)
    _lib.call("hh_tune", b"band4", band4)
    try:
        m = ice.ContactMatrix.from_pixels(b1, b2, c, n, off)
        inf = m.info()
        if band_w > 0:
            assert inf["band_w"] == band_w and inf["band_w4"] == band_w
        if band_w == 0:
            assert inf["band_w"] == 0 and inf["band_w4"] == 0 and inf["n_band"] == 0
        if band_w == -1:
            assert inf["n_band"] > 0  # dense near the diagonal at A=60
            if band4:
                assert inf["band_w4"] > inf["band_w"] and (inf["band_w4"] - inf["band_w"]) % 32 == 0
            else:
                assert inf["band_w4"] == inf["band_w"] > 0
        e1, e2, ec = m.export_upper()
        f1, f2, fc = _filtered_upper(b1, b2, c, off, 1, False)
        np.testing.assert_array_equal(e1, f1)
        np.testing.assert_array_equal(e2, f2)
        np.testing.assert_array_equal(ec, fc)
        w, st = ice.balance_matrix(m)
        m.close()
    finally:
        _lib.call("hh_tune", b"band_w", -1)
        _lib.call("hh_tune", b"band4", 1)
    w_ref, st_ref = ice_ref.balance(b1, b2, c, n, off)
    assert st["iters"] == st_ref["iters"]
    np.testing.assert_allclose(w, w_ref, rtol=1e-9, equal_nan=True)


@pytest.mark.parametrize("upper", [0, 1], ids=["both", "uptiles"])
@pytest.mark.parametrize("flat_max,flat_cols", [(0, -1), (2, -1), (24, -1), (255, -1), (24, 1), (255, 1)])
def test_flat_tiles(ice, flat_max, flat_cols, upper):
    """Tiles whose rows are all short go to the flat (merge-path) sweep kernel;
    any threshold (none, few, most, all tiles flat) gives the oracle's weights,
    and a 3-shard run is bitwise equal to the whole-matrix run -- with both
    triangles in every tile, and with upper-triangle tiles (the column side in
    fixed point, exchanged between the shards as int64)."""
    from hichap_master_amd import _lib
    if upper:
        from tests.shard_exchange import require_uptiles
        require_uptiles()
    b1, b2, c, off = _case(41, sizes=(9000, 7000, 600), A=3.0, trans=0.0005)
    n = int(off[-1])
    _lib.call("hh_tune", b"flat_max", flat_max)
    _lib.call("hh_tune", b"flat_cols", flat_cols)  # 1: the column-grouped kernel (auto: big matrices only)
    _lib.call("hh_tune", b"upper_tiles", upper)
    try:
        m = ice.ContactMatrix.from_pixels(b1, b2, c, n, off)
        inf = m.info()
        if flat_max == 0:
            assert inf["n_units_flat"] == 0
        if flat_max == 255:
            assert inf["n_units_flat"] > 0
        w, st = ice.balance_matrix(m, ice.IceOptions(max_iters=300))
        m.close()
        if upper:
            assert inf["upper"] == 1
        ws, sts = _sharded_weights(ice, b1, b2, c, off, np.array([0, 4096, 11264, n]))
    finally:
        _lib.call("hh_tune", b"flat_max", 64)
        _lib.call("hh_tune", b"flat_cols", -1)
        _lib.call("hh_tune", b"upper_tiles", -1)
    w_ref, st_ref = ice_ref.balance(b1, b2, c, n, off, max_iters=300)
    assert st["iters"] == st_ref["iters"]
    np.testing.assert_allclose(w, w_ref, rtol=1e-9, equal_nan=True)
    np.testing.assert_array_equal(ws, w)
    assert sts["iters"] == st["iters"]


@pytest.mark.parametrize("upper", [0, 1], ids=["both", "uptiles"])
def test_flat_block_shapes_bitwise(ice, upper):
    """The column-grouped flat kernel's block width (waves sharing one staged
    b[J]) and group size (a build knob) change only who sweeps a flat tile,
    not its per-row partials (nor, with upper-triangle tiles, its exact
    fixed-point column partials): bitwise the same weights."""
    from hichap_master_amd import _lib
    if upper:
        from tests.shard_exchange import require_uptiles
        require_uptiles()
    b1, b2, c, off = _case(41, sizes=(9000, 7000, 600), A=3.0, trans=0.0005)
    n = int(off[-1])
    res = []
    _lib.call("hh_tune", b"flat_cols", 1)  # (auto: column groups only from 32 column tiles)
    _lib.call("hh_tune", b"upper_tiles", upper)
    try:
        for waves, group in [(8, 16), (10, 16), (11, 33), (11, 1), (8, 64)]:
            _lib.call("hh_tune", b"flatw_waves", waves)
            _lib.call("hh_tune", b"flatw_waves_up", 11 if waves == 11 else 8)
            _lib.call("hh_tune", b"flat_group", group)
            m = ice.ContactMatrix.from_pixels(b1, b2, c, n, off)
            assert m.info()["n_units_flat"] > 0
            res.append(ice.balance_matrix(m, ice.IceOptions(max_iters=300)))
            m.close()
    finally:
        _lib.call("hh_tune", b"flatw_waves", 11)
        _lib.call("hh_tune", b"flatw_waves_up", 8)
        _lib.call("hh_tune", b"flat_group", 0)
        _lib.call("hh_tune", b"flat_cols", -1)
        _lib.call("hh_tune", b"upper_tiles", -1)
    for w, st in res[1:]:
        np.testing.assert_array_equal(w, res[0][0])
        assert st["iters"] == res[0][1]["iters"]


@pytest.mark.gpu
@pytest.mark.parametrize("cis_only", [0, 1])
def test_flat_interleaved_layout(ice, cis_only):
    """Column-grouped flat tiles are stored interleaved (finalize_flat_layout:
    element k of every lane's run contiguous, so k_sweep_flatw loads them with
    coalesced instructions into the registers the lane-major loads filled).
    The layout exports to the same pixels (the export de-interleaves), the
    weights equal the oracle with the same iterations, and every block shape
    and pipeline depth of k_sweep_flatw gives bitwise the same weights,
    genome-wide and --cis-only (per-chromosome groups converging at
    different iterations).  flat_cols 1 forces column groups on this small
    matrix; the single-launch sweep is never used on such a layout."""
    from hichap_master_amd import _lib
    b1, b2, c, off = _case(43, sizes=(9000, 7000, 600), A=3.0, trans=0.0005)
    n = int(off[-1])
    res = []
    _lib.call("hh_tune", b"flat_cols", 1)
    try:
        for pipe, waves in ((2, 11), (0, 11), (2, 8), (2, 10), (1, 11)):
            _lib.call("hh_tune", b"flatw_pipe", pipe)
            _lib.call("hh_tune", b"flatw_waves", waves)
            m = ice.ContactMatrix.from_pixels(b1, b2, c, n, off, cis_only=cis_only)
            assert m.info()["n_units_flat"] > 0
            if not res:
                e1, e2, ec = m.export_upper()
                f1, f2, fc = _filtered_upper(b1, b2, c, off, 1, cis_only)
                np.testing.assert_array_equal(e1, f1)
                np.testing.assert_array_equal(e2, f2)
                np.testing.assert_array_equal(ec, fc)
            res.append(ice.balance_matrix(m, ice.IceOptions(max_iters=300)))
            m.close()
    finally:
        _lib.call("hh_tune", b"flatw_pipe", 2)
        _lib.call("hh_tune", b"flatw_waves", 11)
        _lib.call("hh_tune", b"flat_cols", -1)
    for w, st in res[1:]:
        np.testing.assert_array_equal(w, res[0][0])
        np.testing.assert_array_equal(st["iters"], res[0][1]["iters"])
    wr, sr = ice_ref.balance(b1, b2, c, n, off, cis_only=bool(cis_only), max_iters=300)
    np.testing.assert_allclose(res[0][0], wr, rtol=1e-9, equal_nan=True)
    np.testing.assert_array_equal(res[0][1]["iters"], sr["iters"])


def _full_config(cfg):
    """Sizes and generator parameters of BASELINE C4 (hg19 diploid 10 kb, 5e9
    pixels, 20 % trans) / C3 (hg19 40 kb, 8e8 pixels, 85 % trans: at 40 kb
    hg19 has only 1.42e8 cis pixels) / C2 (chr1 10 kb, 5e7 pixels)."""
    if cfg == "c4":
        sizes = synth.genome_bins(10000, diploid=True)
        A, td = synth.calibrate(sizes, 5e9, 0.2)
    elif cfg == "c3":
        sizes = synth.genome_bins(40000)
        A, td = synth.calibrate(sizes, 8e8, 0.85)
    else:
        sizes = synth.chrom_bins([synth.HG19["1"]], 10000)
        A, td = synth.calibrate(sizes, 5e7, 0.0)
    return np.asarray(sizes), dict(A=A, trans_density=td, comp_block=200, seed=20201015)


def _windows(cfg, sizes):
    """Three 4096-row windows (512-aligned): the start of chr1, one across a
    chromosome boundary in mid-genome, and (C4) one inside a paternal
    chromosome / (C3) one across the last boundary (chrX)."""
    off = np.concatenate([[0], np.cumsum(sizes)])
    n = int(off[-1])
    al = lambda x: int(max(0, min(n - 4096, x)) // 512 * 512)  # noqa: E731
    mid = off[int(np.searchsorted(off, n // 4))]
    if cfg == "c4":
        p5 = off[len(sizes) // 2 + 4]  # P copy of chr5
        third = al(p5 + 3000)
    else:
        third = al(off[-2] - 2048)
    return [(0, 4096), (al(mid - 2048), al(mid - 2048) + 4096), (third, third + 4096)]


def _window_pixels(sizes, kw, wins):
    """Every pixel of the complete symmetric rows of the windows (bin1 or
    bin2 inside one of them), from the generator's own upper-triangle table
    (hh_synth_pixels: the same counts the layout was built from), streamed
    through HBM in chunks; diagonal pixels excluded (ignore_diags = 1)."""
    import ctypes as C
    import torch
    from hichap_master_amd import ice as hice
    from hichap_master_amd._lib import call
    P = hice.SynthPixels(list(sizes), ordered=False, **kw)
    try:
        n = P.nnz
        chunk = 1 << 28
        buf = [torch.empty(chunk, dtype=torch.int32, device="cuda") for _ in range(3)]
        got = [[], [], []]
        for a in range(0, n, chunk):
            k = min(chunk, n - a)
            for t, src in zip(buf, (P.bin1, P.bin2, P.count)):
                call("hh_device_copy", C.c_void_p(t.data_ptr()), C.c_void_p(src.data_ptr() + 4 * a), 4 * k, None)
            call("hh_synchronize", None)
            b1, b2, c = (t[:k] for t in buf)
            sel = torch.zeros(k, dtype=torch.bool, device="cuda")
            for lo, hi in wins:
                sel |= ((b1 >= lo) & (b1 < hi)) | ((b2 >= lo) & (b2 < hi))
            sel &= b2 > b1
            for g, t in zip(got, (b1, b2, c)):
                g.append(t[sel].cpu().numpy())
            torch.cuda.synchronize()
        return tuple(np.concatenate(g).astype(np.int64) for g in got)
    finally:
        P.close()


def _window_marg(b1, b2, c, w, lo, hi):
    """cooler's marginalize (bincount of count * w[bin1] * w[bin2] over both
    ends) restricted to rows [lo, hi), sequential fp64 (np.bincount)."""
    contrib = c * w[b1] * w[b2]
    m = np.zeros(hi - lo)
    for e in (b1, b2):
        inw = (e >= lo) & (e < hi)
        m += np.bincount(e[inw] - lo, contrib[inw], minlength=hi - lo)
    return m


@pytest.mark.parametrize("cfg", ["c4", "c3"])
def test_full_size_window_marginals(ice, cfg):
    """BASELINE C4 (5e9 pixels) and C3 (8e8) at full size, pinned at the sweep
    level: after k ICE iterations on the whole matrix in
    its production layout (bands, tiled and flat tiles; upper band), the GPU's
    marginal of iteration k + 1 -- marg_i = b_i sum_j A_ij b_j at the GPU's own
    bias b_k -- equals np.bincount over the complete symmetric rows of three
    4096-row windows at rtol 1e-12 (exact up to fp64 summation order).  Then
    ICE runs to convergence and the balanced matrix's marginals over the same
    windows are 1 within the convergence tolerance (var < tol = 1e-5, mean
    within sqrt(tol))."""
    import torch
    sizes, kw = _full_config(cfg)
    n = int(sizes.sum())
    wins = _windows(cfg, sizes)
    m = ice.ContactMatrix.synthetic(list(sizes), **kw)
    inf = m.info()
    assert inf["n_units_flat"] > 0 and inf["n_units"] > inf["n_units_flat"]
    if cfg == "c4":
        assert inf["band_w"] > 0
    st = ice.IceState(m, ice.IceOptions(tol=0.0, max_iters=1 << 30))
    st.marg_local(0)
    st.filter_nnz()
    st.marg_local(1)
    st.filter_count_mad()
    k = 7
    st.run(k)
    assert st.iterations_done() == k
    b = st.bias()
    out = torch.zeros(n, dtype=torch.float64, device="cuda")
    st.marg_local(2, out)
    torch.cuda.synchronize()
    g = out.cpu().numpy()
    st.close()
    w, stc = ice.balance_matrix(m, ice.IceOptions(max_iters=4000))
    m.close()
    assert stc["converged"] and stc["var"] < 1e-5, (stc["var"], stc["iters"])
    b1, b2, c = _window_pixels(sizes, kw, wins)
    # the generator's table is the layout's: rows [0, 4096) as exported
    ms = ice.ContactMatrix.synthetic(list(sizes), row_range=(0, 4096), **kw)
    e1, e2, ec = ms.export_upper()
    ms.close()
    top = b1 < 4096
    np.testing.assert_array_equal(np.stack([b1[top], b2[top], c[top]]), np.stack([e1, e2, ec]))
    wz = np.nan_to_num(w)
    for lo, hi in wins:
        ref = _window_marg(b1, b2, c, b, lo, hi)
        gw = g[lo:hi]
        live = b[lo:hi] > 0
        assert live.sum() > 2048
        np.testing.assert_array_equal(gw[~live], 0.0)
        np.testing.assert_allclose(gw[live], ref[live], rtol=1e-12, atol=0)
        mr = _window_marg(b1, b2, c, wz, lo, hi)[~np.isnan(w[lo:hi])]
        assert abs(mr.mean() - 1.0) < np.sqrt(1e-5), (lo, mr.mean())
        assert mr.var() < 1e-5, (lo, mr.var())


def test_saturated_counts_match_oracle(ice):
    """Counts up to ~1e7 (C3's saturated calibration, A = 1e6, on chr21+22 at
    40 kb: wide-list entries, uint16/uint32 tiles, a dense band): the GPU
    follows cooler's iteration exactly even where it does not converge."""
    sizes = synth.genome_bins(40000, chroms=["21", "22"])
    rng = np.random.default_rng(3)
    b1, b2, c, off = synth.coo_genome(list(sizes), rng, A=1e6, trans_density=0.0557)
    assert c.max() > 65535
    n = int(off[-1])
    w, st = ice.balance(b1, b2, c, n, off, max_iters=60)
    wr, sr = ice_ref.balance(b1, b2, c, n, off, max_iters=60)
    assert st["iters"] == sr["iters"] == 60 and not st["converged"]
    np.testing.assert_allclose(st["var"], sr["var"], rtol=1e-9)
    np.testing.assert_allclose(w, wr, rtol=1e-9, equal_nan=True)


@pytest.mark.parametrize("conc,split,order,fcols", [(1, 0, 0, -1), (1, 1, 0, 1), (1, 1, 1, 1), (1, 0, 1, -1), (1, 1, 2, 1)])
def test_band_concurrent_bitwise(ice, conc, split, order, fcols):
    """Sweep kernels on one stream, or the band sweep / tiled kernel on side
    streams (hh_tune band_concurrent / split_tiles, default on for matrices of
    >= conc_min_bytes of payload; forced here on a small one), launched band
    first or flat first (conc_order), with the plain or the column-grouped
    flat tiles (flat_cols): each kernel writes its own partials, so the
    weights are bitwise equal."""
    from hichap_master_amd import _lib
    b1, b2, c, off = _case(17, sizes=(1500, 900), A=60.0)
    n = int(off[-1])
    _lib.call("hh_tune", b"band_concurrent", 0)
    # the single-launch sweep (auto below 1 GB) is checked before the
    # concurrent one: switch it off so side / side2 really run
    _lib.call("hh_tune", b"sweep_single", 0)
    _lib.call("hh_tune", b"flat_cols", fcols)
    try:
        w0, s0 = ice.balance(b1, b2, c, n, off, max_iters=300)  # one stream
        _lib.call("hh_tune", b"band_concurrent", conc)
        _lib.call("hh_tune", b"split_tiles", split)
        _lib.call("hh_tune", b"conc_order", order)
        _lib.call("hh_tune", b"conc_min_bytes", 0)
        w1, s1 = ice.balance(b1, b2, c, n, off, max_iters=300)
    finally:
        _lib.call("hh_tune", b"band_concurrent", 1)
        _lib.call("hh_tune", b"split_tiles", 1)
        _lib.call("hh_tune", b"conc_order", 1)
        _lib.call("hh_tune", b"conc_min_bytes", 8 << 30)
        _lib.call("hh_tune", b"sweep_single", -1)
        _lib.call("hh_tune", b"flat_cols", -1)
    np.testing.assert_array_equal(w1, w0)
    assert s1["iters"] == s0["iters"]


def test_c1_config_matches_oracle(ice):
    """BASELINE C1 at its own size (one chromosome, 5 000 bins at 40 kb,
    ~2e6 pixels, cooler's 200-iteration cap): GPU == oracle."""
    sizes = [5000]
    A, td = synth.calibrate(sizes, 2e6, 0.0)
    kw = dict(A=A, trans_density=td, comp_block=200, seed=20201015)
    m = ice.ContactMatrix.synthetic(sizes, **kw)
    b1, b2, c = m.export_upper()
    assert 1.5e6 < b1.size < 2.5e6
    w, st = ice.balance_matrix(m, ice.IceOptions(max_iters=200))
    m.close()
    wr, sr = ice_ref.balance(b1, b2, c, 5000, np.array([0, 5000]), max_iters=200)
    assert st["iters"] == sr["iters"] and st["converged"] == sr["converged"]
    np.testing.assert_allclose(w, wr, rtol=1e-9, equal_nan=True)


@pytest.mark.parametrize("cfg", ["c2"])
def test_config_size_balanced_marginals(ice, cfg):
    """BASELINE C2 (hg19 chr1 at 10 kb, 5e7 pixels, cis only) at full size:
    ICE converges and the balanced marginals of the first 4096 rows (complete
    rows: every lower entry of a row < 4096 is in the window), recomputed on
    the host from the exported pixels, are 1 within the tolerance.  (C4 / C3:
    test_full_size_window_marginals.)"""
    if cfg == "c2":
        sizes = synth.chrom_bins([synth.HG19["1"]], 10000)
        A, td = synth.calibrate(sizes, 5e7, 0.0)
    else:
        sizes = synth.genome_bins(40000)
        A, td = synth.calibrate(sizes, 8e8, 0.85)
    kw = dict(A=A, trans_density=td, comp_block=200, seed=20201015)
    m = ice.ContactMatrix.synthetic(sizes, **kw)
    w, st = ice.balance_matrix(m, ice.IceOptions(max_iters=4000))
    m.close()
    assert st["converged"] and st["var"] < 1e-5, (st["var"], st["iters"])
    rows = 4096
    ms = ice.ContactMatrix.synthetic(sizes, row_range=(0, rows), **kw)
    b1, b2, c = ms.export_upper()
    ms.close()
    wz = np.nan_to_num(w)
    contrib = c * wz[b1] * wz[b2]
    marg = np.bincount(b1, contrib, minlength=rows + 1)[:rows] + \
        np.bincount(np.minimum(b2, rows), contrib, minlength=rows + 1)[:rows]
    ok = ~np.isnan(w[:rows])
    assert ok.sum() > rows // 2
    mr = marg[ok]
    assert abs(mr.mean() - 1.0) < np.sqrt(1e-5), mr.mean()
    assert mr.var() < 1e-5, mr.var()


def test_closed_forms(ice):
    """The analytic known answers of tests/test_oracle_ice.py through the HIP
    path: 2 bins (one sweep, var 0, w = 1/sqrt(a)), 3 bins (w0 = sqrt(c/2ab)
    ...), and an all-masked genome-wide matrix (weights NaN, var 0)."""
    from tests.test_oracle_ice import _three_bin
    for a in (1, 7, 123456):
        w, st = ice.balance([0, 0, 1], [0, 1, 1], [5, a, 9], 2, [0, 2], min_nnz=0, mad_max=0)
        np.testing.assert_allclose(w, 1 / np.sqrt(a), rtol=1e-15)
        assert st["iters"] == 1 and st["var"] == 0.0 and st["scale"] == a
    for abc in ((1, 2, 3), (10, 1, 1), (5, 40, 17)):
        (b1, b2, c), w_exact = _three_bin(*abc)
        w, st = ice.balance(b1, b2, c.astype(np.int64), 3, [0, 3], min_nnz=0, mad_max=0, tol=1e-20,
                            max_iters=5000)
        np.testing.assert_allclose(w, w_exact, rtol=1e-8)
    rng = np.random.default_rng(9)
    b1, b2, c, off = synth.coo_genome([40, 30], rng, A=5.0, trans_density=0.0)
    w, st = ice.balance(b1, b2, c, int(off[-1]), off, min_nnz=10 ** 6)
    assert np.isnan(w).all() and st["var"] == 0.0 and np.isnan(st["scale"])


@pytest.mark.parametrize("cis_only", [False, True])
def test_sweep_launch_shapes_bitwise(ice, cis_only):
    """The sweep's launch shapes -- one k_sweep_all launch (small matrices),
    band segments fused or one launch each, 64- or 256-row band blocks --
    produce the same partials: bitwise the same weights and iterations."""
    from hichap_master_amd import _lib
    b1, b2, c, off = _case(23, sizes=(1700, 1100, 600), A=60.0, trans=0.02)
    n = int(off[-1])
    knobs = ("sweep_single", "band_fused", "band_rows", "flat_max")
    default = {"sweep_single": -1, "band_fused": 1, "band_rows": 0, "flat_max": None}
    shapes = [dict(sweep_single=0, band_fused=0, band_rows=256), dict(sweep_single=1),
              dict(sweep_single=0, band_fused=1, band_rows=64), dict(sweep_single=0, band_fused=0, band_rows=64)]
    try:
        ref = None
        for sh in shapes:
            for k in knobs[:3]:
                _lib.call("hh_tune", k.encode(), sh.get(k, default[k]))
            w, st = ice.balance(b1, b2, c, n, off, cis_only=cis_only, max_iters=300)
            if ref is None:
                ref = (w, st)
            np.testing.assert_array_equal(w, ref[0])
            np.testing.assert_array_equal(np.atleast_1d(st["iters"]), np.atleast_1d(ref[1]["iters"]))
    finally:
        for k in knobs[:3]:
            _lib.call("hh_tune", k.encode(), default[k])
    wr, _ = ice_ref.balance(b1, b2, c, n, off, cis_only=cis_only, max_iters=300)
    np.testing.assert_allclose(ref[0], wr, rtol=1e-9, equal_nan=True)


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("cis_only", [False, True])
def test_stats_modes(ice, mode, cis_only):
    """The ICE stats paths (hh_tune fuse_stats: 1 = stats fused into k_marg +
    last-block tails, 2 = tile sums in k_marg then k_stats2 / k_update_big as
    used for matrices of > 128 stats tiles, 0 = never fused: k_stats1
    launched) against the oracle, with the same iteration counts, and
    sharded == one shard bitwise within each mode."""
    from hichap_master_amd import _lib, dist
    b1, b2, c, off = _case(12, sizes=(600, 450, 300))
    n = int(off[-1])
    _lib.call("hh_tune", b"fuse_stats", mode)
    try:
        w, st = ice.balance(b1, b2, c, n, off, cis_only=cis_only, max_iters=400)
        wr, sr = ice_ref.balance(b1, b2, c, n, off, cis_only=cis_only, max_iters=400)
        np.testing.assert_array_equal(np.isnan(w), np.isnan(wr))
        np.testing.assert_allclose(w, wr, rtol=1e-9, equal_nan=True)
        np.testing.assert_array_equal(st["iters"], sr["iters"])
        np.testing.assert_allclose(st["var"], sr["var"], rtol=1e-6, atol=1e-15)
        if not cis_only:
            rr = dist.partition_rows(np.bincount(b1, minlength=n) + np.bincount(b2, minlength=n), 2)
            w0, s0 = _sharded_weights(ice, b1, b2, c, off, rr)
            np.testing.assert_array_equal(w0, w)
            assert s0["iters"] == st["iters"]
    finally:
        _lib.call("hh_tune", b"fuse_stats", -1)
