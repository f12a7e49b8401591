"""cooler drop-in (coolio.py): the cooler v3 schema round trip through the
HDF5 subset, fetch() against a dense build from the pixel table, and (GPU)
``balance_cooler`` = ice.balance / the ICE oracle on the same table, stored
in place as ``bins/weight`` with cooler's attributes.  Parity against
cooler itself is unpinned (cooler / h5py absent)."""
import numpy as np
import pytest

from hichap_master_amd import coolio, h5, synth
from oracle import ice_ref


def _genome(seed=5, res=100000):
    rng = np.random.default_rng(seed)
    chromsizes = [("1", 61_000_000), ("2", 43_500_000), ("X", 25_000_000)]
    nb = [int(np.ceil(L / res)) for _, L in chromsizes]
    b1, b2, c, off = synth.coo_genome(nb, rng, A=30.0, trans_density=0.02)
    return chromsizes, nb, b1, b2, c.astype(np.int32), off


@pytest.fixture
def cool(tmp_path):
    cs, nb, b1, b2, c, off = _genome()
    path = str(tmp_path / "sample.cool")
    cs40 = cs
    g = _genome(7, 400000)
    coolio.create_cooler(path, {100000: (cs, b1, b2, c), 400000: (cs40, g[2], g[3], g[4])},
                         metadata={"onlyIntra": "False"}, assembly="hg19")
    return path, (cs, nb, b1, b2, c, off)


def _dense(b1, b2, c, n):
    M = np.zeros((n, n))
    M[b1, b2] = c
    M[b2, b1] = c
    return M


def test_schema_and_fetch(cool):
    path, (cs, nb, b1, b2, c, off) = cool
    with coolio.Cooler(path + "::100000") as co:
        assert co.chromnames == ["1", "2", "X"]
        assert co.chromsizes == dict(cs)
        assert co.binsize == 100000 and co.info["nnz"] == b1.size and co.info["storage-mode"] == "symmetric-upper"
        np.testing.assert_array_equal(co.chrom_offsets(), off)
        t1, t2, tc = co.pixels_table()
        np.testing.assert_array_equal(t1, b1)
        np.testing.assert_array_equal(t2, b2)
        np.testing.assert_array_equal(tc, c)
        D = _dense(b1, b2, c, int(off[-1]))
        for k, chro in enumerate(co.chromnames):
            lo, hi = int(off[k]), int(off[k + 1])
            M = co.matrix(balance=False).fetch(chro)
            np.testing.assert_array_equal(M, D[lo:hi, lo:hi])
            assert M.dtype == np.int32
        bins = co.bins().fetch("2")
        assert list(bins.columns) == ["chrom", "start", "end"]
        assert bins["end"].iloc[-1] == 43_500_000 and bins["start"].iloc[1] == 100000
    # the enum bins/chrom column and both resolutions
    with h5.File(path) as f:
        assert sorted(f.root.keys()) == ["100000", "400000"]
        d = f["100000/bins/chrom"]
        assert d.type.enum == {"1": 0, "2": 1, "X": 2}
    with coolio.Cooler(path + "::/400000") as co:
        assert co.n_bins == sum(int(np.ceil(L / 400000)) for _, L in cs)


def test_uri_forms(cool):
    path, _ = cool
    assert coolio.parse_uri(path + "::/resolutions/10000") == (path, "resolutions/10000")
    assert coolio.parse_uri(path) == (path, "")


@pytest.mark.gpu
@pytest.mark.parametrize("cis_only", [False, True])
def test_balance_cooler_in_place(cool, cis_only):
    from hichap_master_amd import _lib
    _lib.require_gpu()
    path, (cs, nb, b1, b2, c, off) = cool
    uri = path + "::100000"
    w, st = coolio.balance_cooler(uri, cis_only=cis_only)
    wr, sr = ice_ref.balance(b1, b2, c, int(off[-1]), off, cis_only=cis_only)
    np.testing.assert_allclose(w, wr, rtol=1e-9, equal_nan=True)
    with coolio.Cooler(uri) as co:
        np.testing.assert_array_equal(co.weights(), w)
        a = h5.File(path)["100000/bins/weight"].attrs
        assert a["cis_only"] is cis_only and a["ignore_diags"] == 1 and a["mad_max"] == 5
        assert a["converged"] == st["converged"]
        np.testing.assert_array_equal(np.atleast_1d(a["scale"]), np.atleast_1d(st["scale"]))
        # balanced fetch: w_i w_j count, NaN rows / columns at masked bins
        D = _dense(b1, b2, c, int(off[-1]))
        lo, hi = int(off[0]), int(off[1])
        M = co.matrix(balance=True).fetch("1")
        ref = D[lo:hi, lo:hi] * w[lo:hi, None] * w[None, lo:hi]
        np.testing.assert_allclose(M, ref, rtol=1e-15, equal_nan=True)
        np.testing.assert_array_equal(co.bins().fetch("1")["weight"].values, w[lo:hi])
    # --force: balancing again replaces the column; other resolution untouched
    w2, _ = coolio.balance_cooler(uri, cis_only=not cis_only)
    with coolio.Cooler(uri) as co:
        np.testing.assert_array_equal(co.weights(), w2)
    with coolio.Cooler(path + "::400000") as co:
        assert "weight" not in co._g("bins")


@pytest.mark.gpu
def test_structurefind_from_cooler(cool, tmp_path):
    """StructureFind(cooler_fil, Res).Compartment() / Data_preprocess() read
    the cooler as the reference does (raw for compartments, balanced
    NaN -> 0 for TADs) and equal the in-memory path."""
    from hichap_master_amd import _lib
    from hichap_master_amd.StructureFind import StructureFind
    _lib.require_gpu()
    path, (cs, nb, b1, b2, c, off) = cool
    coolio.balance_cooler(path + "::100000")
    sf = StructureFind(cooler_fil=path, Res=100000)
    comp = sf.Compartment()
    D = _dense(b1, b2, c, int(off[-1]))
    for k, chro in enumerate(["1", "2", "X"]):
        lo, hi = int(off[k]), int(off[k + 1])
        ref = StructureFind(Res=100000).compartment(D[lo:hi, lo:hi])
        np.testing.assert_array_equal(comp[chro], ref)
    out = tmp_path / "pc.txt"
    sf.OutPut_PC_To_txt(str(out))
    lines = out.read_text().splitlines()
    assert len(lines) == int(off[-1]) and lines[0].split("\t")[0] == "1"
    sf.TAD_parameter_init(200000, 4000000, 3, 600000, "ttest")
    sf.Data_preprocess()
    assert sorted(sf.DI_dict) == ["1", "2", "X"]
