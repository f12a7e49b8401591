"""h5.py / coolio.py pinned against the real libhdf5 (HDF5 1.10.6, in
/opt/conda of the build container) at the file-format level (SURVEY.md §8(f)
row 1; reference cooler I/O at /root/reference/HiCHap/matrixBuilding.py:200-205,
:708, StructureFind.py:513, :853, :2006-2015).

* Reading: tests/golden/cooler_{earliest,latest}.cool were written by libhdf5
  itself (tests/golden/make_h5_fixtures.c: cooler's schema as h5py writes it --
  chunked shuffle + gzip-6 tables, vlen UTF-8 attributes, the bins/chrom enum,
  `file::res` groups; the second file with libver "latest": superblock v3, v2
  object headers, dense attribute and link storage, single-chunk / fixed-array
  / extensible-array chunk indexes).  h5.py's listing of each equals the
  listing libhdf5 printed for it (`*.listing.txt`): same tree, types, shapes,
  chunking, filters, values and attributes.
* Writing: files h5.py writes (create_cooler, then the in-place `cooler
  balance --force` append of bins/weight, twice, and enough appends to split
  symbol table nodes) are read back by libhdf5: `h5dump` succeeds, libhdf5's
  listing equals h5.py's, and `h5repack` + `h5diff` find nothing different.
  Skipped where the HDF5 tools are absent (e.g. the GPU box).

cooler's own schema handling (its readers / writers) stays unpinned: cooler
is absent here."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from hichap_master_amd import coolio, h5
from tests.h5_listing import listing

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
H5 = os.environ.get("HDF5_PREFIX", "/opt/conda")
HAVE_H5 = all(os.path.exists(os.path.join(H5, p)) for p in ("include/hdf5.h", "lib/libhdf5.so", "bin/h5dump"))
needs_h5 = pytest.mark.skipif(not HAVE_H5 or shutil.which("gcc") is None, reason="libhdf5 tools absent")


@pytest.fixture(scope="module")
def dumper(tmp_path_factory):
    """The libhdf5 listing tool (make_h5_fixtures.c), built with gcc."""
    exe = str(tmp_path_factory.mktemp("h5bin") / "make_h5_fixtures")
    subprocess.run(["gcc", "-O2", "-I" + os.path.join(H5, "include"), "-o", exe,
                    os.path.join(GOLDEN, "make_h5_fixtures.c"), "-L" + os.path.join(H5, "lib"),
                    "-Wl,-rpath," + os.path.join(H5, "lib"), "-lhdf5"], check=True)
    return exe


def _lib_listing(exe, path):
    r = subprocess.run([exe, "dump", path], capture_output=True, text=True)
    assert r.returncode == 0 and not r.stderr, r.stderr[-2000:]
    return sorted(r.stdout.splitlines())


@pytest.mark.parametrize("name", ["cooler_earliest", "cooler_latest"])
def test_reads_libhdf5_files_exactly(name):
    want = open(os.path.join(GOLDEN, name + ".listing.txt")).read().splitlines()
    got = listing(os.path.join(GOLDEN, name + ".cool"))
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g == w, (g[:160], w[:160])


def _dense_from_pixels(b1, b2, c, lo, hi):
    n = hi - lo
    M = np.zeros((n, n), dtype=c.dtype)
    k = (b1 >= lo) & (b1 < hi) & (b2 < hi)
    M[b1[k] - lo, b2[k] - lo] = c[k]
    M[b2[k] - lo, b1[k] - lo] = c[k]
    return M


@pytest.mark.parametrize("name", ["cooler_earliest", "cooler_latest"])
def test_cooler_reads_on_libhdf5_files(name):
    """The StructureFind reads (StructureFind.py:513, :853, :2006-2010) on
    libhdf5-written coolers: matrix(balance=False / True).fetch(chrom) and
    bins().fetch(chrom)['weight'] against the raw tables."""
    path = os.path.join(GOLDEN, name + ".cool")
    for res in (40000, 500000):
        with coolio.Cooler(f"{path}::{res}") as c:
            assert c.info["format"] == "HDF5::Cooler" and c.info["bin-size"] == res
            assert c.chromnames == ["chr1", "chr22", "chrX"]
            b1, b2, cnt = c.pixels_table()
            assert c.info["nnz"] == b1.size and c.n_bins == c.info["nbins"]
            w = c.weights()
            for ch in c.chromnames:
                lo, hi = c.extent(ch)
                raw = c.matrix(balance=False).fetch(ch)
                np.testing.assert_array_equal(raw, _dense_from_pixels(b1, b2, cnt, lo, hi))
                bal = c.matrix(balance=True).fetch(ch)
                want = raw * np.outer(w[lo:hi], w[lo:hi])
                np.testing.assert_array_equal(np.isnan(bal), np.isnan(want))
                np.testing.assert_allclose(bal, want, rtol=1e-15, equal_nan=True)
                np.testing.assert_array_equal(c.bins().fetch(ch)["weight"].to_numpy(), w[lo:hi])
        with h5.File(path) as f:
            a = f[f"{res}/bins/weight"].attrs
            assert a["cis_only"] is (res == 500000) and a["divisive_weights"] is False
            assert a["ignore_diags"] == 1 and a["mad_max"] == 5


def test_append_refused_on_latest_format(tmp_path):
    """In-place appends are limited to superblock v0/v1 files (what h5py and
    cooler write by default); a libver-latest file raises instead of being
    corrupted."""
    p = str(tmp_path / "l.cool")
    shutil.copy(os.path.join(GOLDEN, "cooler_latest.cool"), p)
    before = open(p, "rb").read()
    with pytest.raises(h5.H5Error):
        h5.append_dataset(p, "40000/bins", "weight", np.zeros(111))
    assert open(p, "rb").read() == before


def _written_cooler(path):
    rng = np.random.default_rng(5)
    chroms = [("chr1", 2_000_000), ("chr22", 1_500_000), ("chrX", 900_000)]
    res = {}
    for binsize in (40000, 500000):
        nb = sum(-(-L // binsize) for _, L in chroms)
        i, j = np.triu_indices(nb)
        keep = rng.random(i.size) < 0.3
        c = rng.integers(1, 500, size=keep.sum()).astype(np.int32)
        res[binsize] = (chroms, i[keep], j[keep], c)
    coolio.create_cooler(path, res, metadata={"note": "été"}, assembly="hg19")
    return res


def _balance_like_appends(path):
    """What balance_cooler writes (bins/weight + cooler's attributes), twice
    as --force re-runs do, plus a second column name."""
    for res, cis in ((40000, False), (500000, True)):
        with coolio.Cooler(f"{path}::{res}") as c:
            nb = c.n_bins
        w = np.linspace(0.5, 2.0, nb)
        w[::7] = np.nan
        attrs = {"tol": 1e-5, "min_nnz": 10, "min_count": 0, "mad_max": 5, "cis_only": cis, "ignore_diags": 1,
                 "converged": np.array([True, False, True]) if cis else True,
                 "var": np.array([1e-6, 2e-5, 3e-7]) if cis else 4e-6,
                 "scale": np.array([10.5, 20.25, 3.0]) if cis else 123.5, "divisive_weights": False}
        h5.append_dataset(path, f"{res}/bins", "weight", w * 3, attrs)
        h5.append_dataset(path, f"{res}/bins", "weight", w, attrs)  # --force
        h5.append_dataset(path, f"{res}/bins", "weight_cis", w[::-1].copy(), {"cis_only": True})


@needs_h5
def test_libhdf5_reads_written_cooler(tmp_path, dumper):
    p = str(tmp_path / "w.cool")
    _written_cooler(p)
    assert _lib_listing(dumper, p) == listing(p)
    _balance_like_appends(p)
    lib = _lib_listing(dumper, p)
    assert lib == listing(p)
    assert any(x.startswith("A /40000@format vstr") for x in lib)  # str attributes as h5py stores them
    assert any(x.startswith("D /40000/bins/chrom enum(i4){chr1=0,chr22=1,chrX=2}") for x in lib)
    r = subprocess.run([os.path.join(H5, "bin", "h5dump"), "-H", p], capture_output=True, text=True)
    assert r.returncode == 0 and "error" not in (r.stdout + r.stderr).lower(), r.stderr[-2000:]
    q = str(tmp_path / "repacked.cool")
    subprocess.run([os.path.join(H5, "bin", "h5repack"), p, q], check=True, capture_output=True)
    r = subprocess.run([os.path.join(H5, "bin", "h5diff"), p, q], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


@needs_h5
def test_libhdf5_reads_split_symbol_table_nodes(tmp_path, dumper):
    """Appends past a symbol table node's capacity (8) split the node, as
    libhdf5 does: libhdf5 still lists every link, in name order."""
    p = str(tmp_path / "s.h5")
    h5.write_file(p, {"bins": {"start": np.arange(6), "end": np.arange(6) + 1}})
    names = [f"col{k:02d}" for k in range(37)] + ["a", "zzz"]
    for k, nm in enumerate(names):
        h5.append_dataset(p, "bins", nm, np.full(3, k, dtype=np.int64))
    lib = _lib_listing(dumper, p)
    assert lib == listing(p)
    assert sum(1 for x in lib if x.startswith("D /bins/")) == len(names) + 2


@needs_h5
def test_append_into_libhdf5_file(tmp_path, dumper):
    """`cooler balance --force` onto a file libhdf5 wrote: bins/weight
    replaced and a new column added in place; libhdf5 and h5.py agree."""
    p = str(tmp_path / "e.cool")
    shutil.copy(os.path.join(GOLDEN, "cooler_earliest.cool"), p)
    _balance_like_appends(p)
    lib = _lib_listing(dumper, p)
    assert lib == listing(p)
    with h5.File(p) as f:
        w = f["40000/bins/weight"].read()
        assert np.isnan(w[0]) and w[1] == np.linspace(0.5, 2.0, 111)[1]
        assert "weight_cis" in f["500000/bins"].keys()
