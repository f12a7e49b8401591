"""Pair binning on the GPU (hh_binner_* through the C-ABI) against the
reference's golden outputs and the CPU oracle (oracle/pairs_ref.py).
Counts are integers: every comparison is exact."""
import json

import numpy as np
import pytest

from oracle import pairs_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mb():
    from hichap_master_amd import _lib, matrixBuilding
    _lib.require_gpu()
    return matrixBuilding


def _bytes(a):
    return bytes(np.asarray(a, dtype=np.uint8))


def _lines(a):
    return _bytes(a).decode().splitlines(keepends=True)


def _golden_keys(g, prefix):
    out = {}
    for k in g:
        if k.startswith(prefix + "/"):
            _, res, key, f = k.split("/")
            out.setdefault((int(res), key), {})[f] = g[k]
    return out


def _genome_file(tmp_path, g):
    p = tmp_path / "genome.txt"
    p.write_bytes(_bytes(g["genome"]))
    return str(p)


@pytest.mark.parametrize("case", ["pairs_traditional", "pairs_traditional_allchroms"])
@pytest.mark.parametrize("how", ["bytes", "lines", "file_small_chunks"])
def test_traditional_matches_reference(mb, golden, tmp_path, case, how):
    g = golden(case)
    p = json.loads(str(g["params"]))
    gpath = _genome_file(tmp_path, g)
    if how == "bytes":
        src = _bytes(g["text"])
    elif how == "lines":
        src = _lines(g["text"])
    else:
        f = tmp_path / "Sample_Valid.bed"
        f.write_bytes(_bytes(g["text"]))
        src = str(f)
    if how == "file_small_chunks":
        from hichap_master_amd import pairs
        old = pairs.CHUNK_BYTES
        pairs.CHUNK_BYTES = 4096  # many chunks: lines cut across block and device-chunk boundaries
        try:
            W, L = mb.TraditionalMatrixBuilding(src, gpath, p["wholeRes"], p["localRes"], p["chroms"])
        finally:
            pairs.CHUNK_BYTES = old
    else:
        W, L = mb.TraditionalMatrixBuilding(src, gpath, p["wholeRes"], p["localRes"], p["chroms"])
    for prefix, lib in (("whole", W), ("local", L)):
        gk = _golden_keys(g, prefix)
        got = {(res, key): arr for res, d in lib.items() for key, arr in d.items()}
        assert set(got) == set(gk)
        for k, arr in got.items():
            assert arr.dtype == pairs_ref._SD
            for f in ("bin1", "bin2", "IF"):
                np.testing.assert_array_equal(arr[f], gk[k][f], err_msg=f"{k} {f}")


def _check_dense(gk, whole_lib, local_lib):
    for (res, key), d in gk.items():
        M = whole_lib[res]["Matrix"] if key == "__whole__" else local_lib[res][key]
        assert M.dtype == np.int64 and (M == M.T).all()
        i, j = np.nonzero(np.triu(M))
        np.testing.assert_array_equal(i, d["bin1"])
        np.testing.assert_array_equal(j, d["bin2"])
        np.testing.assert_array_equal(M[i, j].astype(np.float64), d["IF"])


def test_allelic_traditional_matches_reference(mb, golden, tmp_path):
    g = golden("pairs_allelic_traditional")
    p = json.loads(str(g["params"]))
    W, L = mb.TraditionalMatrixInAllelic(_bytes(g["text"]), _genome_file(tmp_path, g), p["wholeRes"],
                                         p["localRes"], p["chroms"])
    gk = _golden_keys(g, "whole")
    gk.update(_golden_keys(g, "local"))
    _check_dense(gk, W, L)


def test_haplotype_unimputed_matches_reference(mb, golden, tmp_path):
    g = golden("pairs_haplotype_unimputed")
    p = json.loads(str(g["params"]))
    src = {k: _bytes(g["text_" + k]) for k in ("M_M", "P_P", "M_P", "P_M")}
    UW, UL = mb.HaplotypeUnImputedBuilding(src["M_M"], src["P_P"], src["M_P"], src["P_M"],
                                           _genome_file(tmp_path, g), p["wholeRes"], p["localRes"], p["chroms"])
    gk = _golden_keys(g, "whole")
    gk.update(_golden_keys(g, "local"))
    _check_dense(gk, UW, UL)


# ----------------------------------------------------------- larger, vs oracle
GENOME = {"1": 24_925_062, "2": 24_319_237, "3": 19_802_243, "X": 15_527_060}


def _synth_text(n, seed, fmt=0):
    """Device-generated synthetic pair text (hh_synth_pairs_text) copied to the host."""
    import ctypes as C
    import torch
    from hichap_master_amd._lib import call
    names = b"".join(b"chr" + c.encode() + b"\0" for c in GENOME)
    lens = np.array(list(GENOME.values()), dtype=np.int64)
    nb = C.c_int64(0)
    call("hh_synth_pairs_text", len(GENOME), names, lens.ctypes.data_as(C.c_void_p), n, 0.8, 2e6, fmt, seed, 0,
         None, 0, C.byref(nb), None)
    buf = torch.empty(nb.value, dtype=torch.uint8, device="cuda")
    call("hh_synth_pairs_text", len(GENOME), names, lens.ctypes.data_as(C.c_void_p), n, 0.8, 2e6, fmt, seed, 0,
         C.c_void_p(buf.data_ptr()), nb.value, C.byref(nb), None)
    torch.cuda.synchronize()
    return buf, bytes(buf.cpu().numpy())


def test_synthetic_many_chunks_vs_oracle(mb):
    from hichap_master_amd import pairs
    buf, text = _synth_text(120_000, 5)
    lines = text.decode().splitlines(keepends=True)
    assert len(lines) == 120_000
    chroms = ["#", "X"]
    whole, local = pairs_ref.traditional_counts(lines, GENOME, chroms, [1_000_000, 250_000], [100_000])
    B = pairs.PairBinner(GENOME, chroms)
    tw = B.add_target(1_000_000)
    tw2 = B.add_target(250_000)
    tl = B.add_target(100_000, local=True)
    B.feed(text, pairs.pairs_format(pairs.VALID_BED), chunk_bytes=1 << 20)  # ~14 device chunks
    st = B.stats()
    assert st["lines"] == 120_000 and st["binned"] == 120_000
    for t, counter in ((tw, whole[1_000_000]), (tw2, whole[250_000])):
        b1, b2, c = B.pixels(t)
        e1, e2, ec = pairs_ref.counter_to_pixels(counter)
        np.testing.assert_array_equal(b1, e1)
        np.testing.assert_array_equal(b2, e2)
        np.testing.assert_array_equal(c, ec)
    b1, b2, c = B.pixels(tl)
    order = pairs.sort_chromosomes(GENOME)
    lsd = pairs.local_sparse_dict(b1, b2, c, tl, order)
    for chro in order:
        e1, e2, ec = pairs_ref.counter_to_pixels(local[100_000][chro])
        np.testing.assert_array_equal(lsd[chro]["bin1"], e1)
        np.testing.assert_array_equal(lsd[chro]["bin2"], e2)
        np.testing.assert_array_equal(lsd[chro]["IF"], ec.astype(np.float64))
    # the device-resident path (bench input) gives the same tables
    B2 = pairs.PairBinner(GENOME, chroms)
    t2 = B2.add_target(1_000_000)
    B2.feed_device(buf.data_ptr(), buf.numel(), pairs.pairs_format(pairs.VALID_BED))
    for a, b in zip(B2.pixels(t2), B.pixels(tw)):
        np.testing.assert_array_equal(a, b)
    B.close()
    B2.close()


def test_allelic_synthetic_mark_filter_vs_oracle(mb):
    from hichap_master_amd import pairs
    _, text = _synth_text(40_000, 9, fmt=1)
    lines = text.decode().splitlines(keepends=True)
    src = {"M_M": lines[:20000], "P_P": lines[20000:30000], "M_P": lines[30000:35000], "P_M": lines[35000:]}
    whole, local = pairs_ref.haplotype_counts(src, GENOME, ["#", "X"], [500_000], [200_000])
    UW, UL = mb.HaplotypeUnImputedBuilding(*("".join(src[k]).encode() for k in ("M_M", "P_P", "M_P", "P_M")),
                                           _GenomeLines(GENOME), [500_000], [200_000], ["#", "X"], dense=False)
    b1, b2, c = UW[500_000]["Matrix"]
    e1, e2, ec = pairs_ref.counter_to_pixels(whole[500_000])
    np.testing.assert_array_equal(b1, e1)
    np.testing.assert_array_equal(b2, e2)
    np.testing.assert_array_equal(c, ec)
    for key, counter in local[200_000].items():
        x, y, v = UL[200_000][key]
        e1, e2, ec = pairs_ref.counter_to_pixels(counter)
        np.testing.assert_array_equal(x, e1)
        np.testing.assert_array_equal(y, e2)
        np.testing.assert_array_equal(v, ec)


class _GenomeLines(list):
    def __init__(self, genome):
        super().__init__(f"chr{c}\t{l}\n" for c, l in genome.items())


# ----------------------------------------------------------- edge cases
def _run(text, genome=None, chroms=("#", "X"), whole=(100000,), local=(), fmt=None):
    from hichap_master_amd import pairs
    genome = genome or {"1": 1_000_000, "2": 500_000}
    B = pairs.PairBinner(genome, list(chroms))
    ts = [B.add_target(r) for r in whole] + [B.add_target(r, local=True) for r in local]
    try:
        B.feed(text, fmt or pairs.pairs_format(pairs.VALID_BED))
        return B.stats(), [B.pixels(t) for t in ts]
    finally:
        B.close()


OK = b"r chr1 + 5 0 0 100 0 chr2 - 5 0 0 200 0\n"


def test_empty_and_whitespace_inputs(mb):
    st, px = _run(b"")
    assert st["lines"] == 0 and px[0][0].size == 0
    st, px = _run(OK * 3 + OK.rstrip(b"\n"))  # final line without newline
    assert st["lines"] == 4 and px[0][2].tolist() == [4]
    st, px = _run(OK.replace(b"\n", b"\r\n").replace(b" ", b" \t "))
    assert st["binned"] == 1


@pytest.mark.parametrize("bad,msg", [
    (b"\n", "missing field"),                                       # empty line: line[1] IndexError
    (b"r chr1 + 5 0 0 100 0 chr2\n", "missing field"),               # no field 13
    (OK.replace(b" 100 ", b" 1e2 "), "integer"),                      # int('1e2') ValueError
    (OK.replace(b" 100 ", b" -100 "), "integer"),                     # negative: would wrap in NumPy
    (OK.replace(b"chr2", b"chr3"), "KeyError"),                       # passes '#', not in genome
    (OK.replace(b" 200 ", b" 900000 "), "bin outside"),               # past the whole matrix
])
def test_lines_the_reference_rejects_raise(mb, bad, msg):
    from hichap_master_amd._lib import HipLibraryError
    with pytest.raises(HipLibraryError, match=msg) as e:
        _run(OK * 5 + bad + OK)
    assert "pair line 6" in str(e.value)


def test_filters_and_quirks(mb):
    # chrY fails ['#', 'X'] -> skipped even if its other fields are garbage
    st, px = _run(OK + b"r chrY + 5 0 0 zz 0 chr1 - 5 0 0 200 0\n")
    assert st["skipped_chrom"] == 1 and px[0][2].sum() == 1
    # 'chr' is lstripped as a character set: "chrchr1" and "rhc1" are chromosome 1
    st, px = _run(OK.replace(b"chr1", b"chrchr1") + OK.replace(b"chr1", b"rhc1"))
    assert st["binned"] == 2
    # position past the chromosome end but inside the whole matrix spills into
    # the next chromosome's bins (the reference's dense indexing does the same)
    st, px = _run(OK.replace(b" 100 ", b" 1200000 "))
    assert px[0][0].tolist() == [11] and px[0][1].tolist() == [12]
    # ... but raises for an intra-chromosome (local) matrix
    from hichap_master_amd._lib import HipLibraryError
    with pytest.raises(HipLibraryError, match="bin outside"):
        _run(OK.replace(b" 100 ", b" 1200000 ").replace(b"chr2", b"chr1"), local=(100000,))
    # trans pairs never reach an intra-chromosome matrix; no whole target: a
    # trans line's positions are never parsed (as in the reference)
    st, px = _run(OK.replace(b" 100 ", b" x "), whole=(), local=(50000,))
    assert px[0][0].size == 0
    # empty chroms list: everything in the genome passes, unknown names raise
    with pytest.raises(HipLibraryError, match="KeyError"):
        _run(OK.replace(b"chr2", b"chrUn"), chroms=())


def test_mark_filter(mb):
    from hichap_master_amd import pairs
    f = pairs.pairs_format(pairs.ALLELIC_BED, "Both")
    text = b"chr1 5 chr1 900 Both\nchr1 5 chr1 900 R1\nchr1 7 chr1 1000 Both\n"
    st, px = _run(text, fmt=f)
    assert st["skipped_mark"] == 1 and px[0][2].tolist() == [2]
    from hichap_master_amd._lib import HipLibraryError
    with pytest.raises(HipLibraryError, match="missing field"):
        _run(text + b"\n", fmt=f)  # line[-1] of an empty line


def test_ice_on_binned_pixels(mb):
    """Pair text -> GPU binning -> GPU ICE equals the oracle chain."""
    from hichap_master_amd import ice, pairs
    from oracle import ice_ref
    _, text = _synth_text(200_000, 11)
    lines = text.decode().splitlines(keepends=True)
    whole, _ = pairs_ref.traditional_counts(lines, GENOME, ["#", "X"], [500_000], [])
    e1, e2, ec = pairs_ref.counter_to_pixels(whole[500_000])
    B = pairs.PairBinner(GENOME, ["#", "X"])
    t = B.add_target(500_000)
    B.feed(text, pairs.pairs_format(pairs.VALID_BED))
    b1, b2, c = B.pixels(t)
    B.close()
    off = np.concatenate([[0], np.cumsum(t.chrom_nbins)]).astype(np.int64)
    w, st = ice.balance(b1.astype(np.int64), b2.astype(np.int64), c.astype(np.float64), int(off[-1]), off)
    w_ref, st_ref = ice_ref.balance(e1, e2, ec.astype(np.float64), int(off[-1]), off)
    assert st["iters"] == st_ref["iters"]
    np.testing.assert_allclose(w, w_ref, rtol=1e-9, equal_nan=True)


def test_long_lines_and_unaligned_device_text(mb):
    """Lines far longer than a tile's 1 KB lookahead (fields read through the
    global fallback), and device text starting at an unaligned address."""
    import torch
    from hichap_master_amd import pairs
    rng = np.random.default_rng(21)
    names = ["chr1", "chr2", "chr3", "chrX", "chrY"]
    out = []
    for k in range(3000):
        c1, c2 = names[rng.integers(5)], names[rng.integers(5)]
        p1, p2 = int(rng.integers(0, 15_000_000)), int(rng.integers(0, 15_000_000))
        pad = "x" * int(rng.choice([1, 50, 3000, 9000], p=[0.6, 0.3, 0.07, 0.03]))
        sep = " " * int(rng.integers(1, 4))
        out.append(sep.join([f"R{k}{pad}", c1, "+", str(p1), "0", "0", str(p1), "0", c2, "-", str(p2), "0", "0",
                             str(p2), "0" + pad]) + "\n")
    text = "".join(out).encode()
    lines = text.decode().splitlines(keepends=True)
    whole, local = pairs_ref.traditional_counts(lines, GENOME, ["#", "X"], [500_000], [250_000])
    for shift in (0, 3, 13):
        buf = torch.zeros(len(text) + 32, dtype=torch.uint8, device="cuda")
        buf[shift:shift + len(text)] = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
        B = pairs.PairBinner(GENOME, ["#", "X"])
        tw = B.add_target(500_000)
        tl = B.add_target(250_000, local=True)
        B.feed_device(buf.data_ptr() + shift, len(text), pairs.pairs_format(pairs.VALID_BED))
        b1, b2, c = B.pixels(tw)
        e1, e2, ec = pairs_ref.counter_to_pixels(whole[500_000])
        np.testing.assert_array_equal(b1, e1)
        np.testing.assert_array_equal(b2, e2)
        np.testing.assert_array_equal(c, ec)
        lsd = pairs.local_sparse_dict(*B.pixels(tl), tl, pairs.sort_chromosomes(GENOME))
        for chro in lsd:
            e1, e2, ec = pairs_ref.counter_to_pixels(local[250_000][chro])
            np.testing.assert_array_equal(lsd[chro]["bin2"], e2)
            np.testing.assert_array_equal(lsd[chro]["IF"], ec.astype(np.float64))
        assert B.stats()["lines"] == 3000
        B.close()
