"""Device build of the ICE layout from cooler's pixel table (build.hip,
hh_matrix_from_pixels_device) against the host builder: identical layout
(export round trip, counts, bands), identical ICE weights (bitwise: same plan
=> same summation order), the reference's filter semantics, and loud errors.
Reference: the `cooler balance` inputs of matrixBuilding.py:699-714."""
import numpy as np
import pytest

from hichap_master_amd import synth
from oracle import ice_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ice():
    from hichap_master_amd import _lib, ice
    _lib.require_gpu()
    return ice


def _host_build(ice, *a, **kw):
    from hichap_master_amd._lib import call
    call("hh_tune", b"host_build", 1)
    try:
        return ice.ContactMatrix.from_pixels(*a, **kw)
    finally:
        call("hh_tune", b"host_build", 0)


def _same_matrix(ice, m1, m2):
    i1, i2 = m1.info(), m2.info()
    for k in ("n_bins", "row_lo", "row_hi", "nnz_upper", "n_entries", "n_slots", "n_slots_narrow", "n_tiles",
              "n_units", "n_wide", "payload_bytes", "band_w", "band_w4", "n_band", "n_units_flat"):
        assert i1[k] == i2[k], (k, i1[k], i2[k])
    for a, b in zip(m1.export_upper(), m2.export_upper()):
        np.testing.assert_array_equal(a, b)


def _genome(seed, sizes=(900, 700, 500), A=30.0, trans=0.01, big=False):
    rng = np.random.default_rng(seed)
    b1, b2, c, off = synth.coo_genome(list(sizes), rng, A=A, trans_density=trans)
    c = c.astype(np.int64)
    if big:  # counts for the uint8 / 4-bit bands' limits and the wide list
        k = rng.choice(c.size, size=60, replace=False)
        c[k[:20]] = rng.integers(256, 60000, size=20)
        c[k[20:40]] = rng.integers(65536, 2_000_000, size=20)
        c[k[40:]] = rng.integers(16, 255, size=20)
    return b1, b2, c, off


@pytest.fixture
def upper_tiles():
    """upper-triangle tiles forced on (the 4096-column build
    only); auto afterwards"""
    from hichap_master_amd._lib import call
    from tests.shard_exchange import require_uptiles
    require_uptiles()
    call("hh_tune", b"upper_tiles", 1)
    yield
    call("hh_tune", b"upper_tiles", -1)


@pytest.mark.parametrize("ignore_diags,cis_only,big", [(1, False, False), (0, False, True), (2, True, False),
                                                       (1, True, True)])
def test_device_build_equals_host_build(ice, ignore_diags, cis_only, big):
    b1, b2, c, off = _genome(3 + ignore_diags, big=big)
    n = int(off[-1])
    md = ice.ContactMatrix.from_pixels(b1, b2, c, n, off, ignore_diags, cis_only)
    mh = _host_build(ice, b1, b2, c, n, off, ignore_diags, cis_only)
    _same_matrix(ice, md, mh)
    opts = ice.IceOptions(ignore_diags=ignore_diags, cis_only=cis_only, max_iters=300)
    wd, sd = ice.balance_matrix(md, opts)
    wh, sh = ice.balance_matrix(mh, opts)
    np.testing.assert_array_equal(wd, wh)
    np.testing.assert_array_equal(np.atleast_1d(sd["iters"]), np.atleast_1d(sh["iters"]))
    w_ref, st_ref = ice_ref.balance(b1, b2, c, n, off, ignore_diags=ignore_diags, cis_only=cis_only, max_iters=300)
    np.testing.assert_allclose(wd, w_ref, rtol=1e-9, equal_nan=True)


@pytest.mark.parametrize("ignore_diags,cis_only,big", [(1, False, True), (2, True, False)])
def test_device_build_equals_host_build_uptiles(ice, upper_tiles, ignore_diags, cis_only, big):
    """The same with upper-triangle tiles: both builders keep an entry of a
    lower tile only as its mirror; weights bitwise equal, the oracle's within
    the ICE tolerance, and close to the both-triangle layout: the column
    side rounds b to b * 2^e (e from the raw-marginal bound; counts to 2e6
    here cost ~22 bits of it), so up to ~1e-11 of a converged weight."""
    from hichap_master_amd._lib import call
    b1, b2, c, off = _genome(13 + ignore_diags, sizes=(5000, 4000, 700), big=big)
    n = int(off[-1])
    md = ice.ContactMatrix.from_pixels(b1, b2, c, n, off, ignore_diags, cis_only)
    mh = _host_build(ice, b1, b2, c, n, off, ignore_diags, cis_only)
    assert md.info()["upper"] == 1 and mh.info()["upper"] == 1
    _same_matrix(ice, md, mh)
    opts = ice.IceOptions(ignore_diags=ignore_diags, cis_only=cis_only, max_iters=300)
    wd, sd = ice.balance_matrix(md, opts)
    wh, sh = ice.balance_matrix(mh, opts)
    np.testing.assert_array_equal(wd, wh)
    np.testing.assert_array_equal(np.atleast_1d(sd["iters"]), np.atleast_1d(sh["iters"]))
    call("hh_tune", b"upper_tiles", 0)
    mb = ice.ContactMatrix.from_pixels(b1, b2, c, n, off, ignore_diags, cis_only)
    assert mb.info()["upper"] == 0 and mb.info()["payload_bytes"] > md.info()["payload_bytes"]
    wb, sb = ice.balance_matrix(mb, opts)
    np.testing.assert_array_equal(np.atleast_1d(sd["iters"]), np.atleast_1d(sb["iters"]))
    np.testing.assert_allclose(wd, wb, rtol=1e-12 if not big else 1e-10, equal_nan=True)
    w_ref, st_ref = ice_ref.balance(b1, b2, c, n, off, ignore_diags=ignore_diags, cis_only=cis_only, max_iters=300)
    np.testing.assert_allclose(wd, w_ref, rtol=1e-9, equal_nan=True)


def test_device_build_shards(ice):
    b1, b2, c, off = _genome(11, sizes=(1400, 900, 600), trans=0.02)
    n = int(off[-1])
    mh = _host_build(ice, b1, b2, c, n, off)
    for lo, hi in [(0, 512), (512, 1536), (1536, n)]:
        md = ice.ContactMatrix.from_pixels(b1, b2, c, n, off, row_range=(lo, hi))
        mhs = _host_build(ice, b1, b2, c, n, off, row_range=(lo, hi))
        _same_matrix(ice, md, mhs)
    assert mh.info()["nnz_upper"] > 0


def test_unsorted_and_lower_triangle_fall_back_to_host(ice):
    b1, b2, c, off = _genome(5)
    n = int(off[-1])
    ref = ice.ContactMatrix.from_pixels(b1, b2, c, n, off)
    rng = np.random.default_rng(0)
    p = rng.permutation(b1.size)
    flip = rng.random(b1.size) < 0.3
    x1, x2 = np.where(flip, b2, b1)[p], np.where(flip, b1, b2)[p]
    m = ice.ContactMatrix.from_pixels(x1, x2, c[p], n, off)
    _same_matrix(ice, m, ref)


def test_device_pixels_api_and_errors(ice):
    import torch
    from hichap_master_amd._lib import HipLibraryError
    b1, b2, c, off = _genome(7)
    n = int(off[-1])
    ref = ice.ContactMatrix.from_pixels(b1, b2, c, n, off)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).cuda()
    m = ice.ContactMatrix.from_device_pixels(t(b1), t(b2), t(c), n, off)
    _same_matrix(ice, m, ref)
    # duplicate pixel
    d1, d2, dc = np.insert(b1, 10, b1[10]), np.insert(b2, 10, b2[10]), np.insert(c, 10, 1)
    with pytest.raises(HipLibraryError, match="duplicate"):
        ice.ContactMatrix.from_device_pixels(t(d1), t(d2), t(dc), n, off)
    with pytest.raises(HipLibraryError, match="duplicate"):
        ice.ContactMatrix.from_pixels(d1, d2, dc, n, off)
    # out of order on the device API (no fallback there)
    with pytest.raises(HipLibraryError, match="sorted"):
        ice.ContactMatrix.from_device_pixels(t(b1[::-1]), t(b2[::-1]), t(c[::-1]), n, off)
    # id out of range / negative count
    e2 = b2.copy()
    e2[-1] = n
    with pytest.raises(HipLibraryError, match="range"):
        ice.ContactMatrix.from_device_pixels(t(b1), t(e2), t(c), n, off)
    ec = c.copy()
    ec[5] = -1
    with pytest.raises(HipLibraryError, match="non-negative"):
        ice.ContactMatrix.from_device_pixels(t(b1), t(b2), t(ec), n, off)


def test_empty_table(ice):
    off = np.array([0, 600, 1000])
    e = np.zeros(0, np.int64)
    m = ice.ContactMatrix.from_pixels(e, e, e, 1000, off)
    assert m.info()["nnz_upper"] == 0
    w, st = ice.balance_matrix(m)
    assert np.isnan(w).all()


def test_pair_binner_to_contact_matrix(ice):
    """PairBinner -> ContactMatrix on the device (no host copy of the pixel
    table) equals building from the downloaded table, and balances the same."""
    import torch
    from hichap_master_amd import pairs
    from bench import synth_pairs_text
    genome = {"1": 40_000_000, "2": 30_000_000, "3": 20_000_000}
    text = synth_pairs_text(genome, 400_000, seed=3)
    B = pairs.PairBinner(genome, ["#", "X"], stream=torch.cuda.current_stream().cuda_stream)
    tw = B.add_target(100000)
    tl = B.add_target(100000, local=True)
    B.feed_device(text.data_ptr(), text.numel(), pairs.pairs_format(pairs.VALID_BED))
    B.finish()
    for t in (tw, tl):
        m = B.contact_matrix(t)
        b1, b2, c = B.pixels(t)
        ref = ice.ContactMatrix.from_pixels(b1, b2, c, t.n_bins, B.chrom_offsets(t), 1, t.local)
        _same_matrix(ice, m, ref)
        opts = ice.IceOptions(cis_only=t.local, max_iters=300)
        np.testing.assert_array_equal(ice.balance_matrix(m, opts)[0], ice.balance_matrix(ref, opts)[0])
    B.close()
