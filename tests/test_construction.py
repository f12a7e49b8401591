"""The `hichap matrix` drop-in (matrixBuilding.py:617-717, :1495-1860):
NPZ2Cooler's pixel tables, replicate merging and in-place balancing of the
multi-resolution coolers.

CPU: NPZ2Cooler on the reference's own sparse dicts (tests/golden/
pairs_traditional.npz, the reference's TraditionalMatrixBuilding output) gives
the oracle's tables (oracle/cooler_ref.py, the reference's `_generator`
restated with scipy.sparse as it is written); the file is a cooler that
coolio reads back and libhdf5 lists (h5dump-style), merge_coolers sums
replicates; an asymmetric intra block follows the reference's lil
symmetrisation.  GPU: TraditionalMatrixConstruction from the golden Valid.bed
text (two replicates) -> replicate + merged coolers whose tables equal the
oracle's and whose weights equal the oracle ICE (cooler balance: genome-wide
for wholeRes, --cis-only for localRes) on the same tables; and
HaplotypeMatrixConstruction from the golden allelic beds."""
import json
import os

import numpy as np
import pytest

from oracle import cooler_ref, ice_ref

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _libs(g, p):
    W, L = {}, {}
    for k in g:
        part = k.split("/")
        if len(part) == 4 and part[0] in ("whole", "local"):
            kind, res, key, fld = part
            d = (W if kind == "whole" else L).setdefault(int(res), {})
            d.setdefault(key, {})[fld] = g[k]
    def cvt(lib):
        return {res: {key: _rec(v) for key, v in d.items()} for res, d in lib.items()}
    return cvt(W), cvt(L)


def _rec(v):
    t = np.zeros(v["bin1"].size, dtype=cooler_ref.S_DTYPE)
    t["bin1"], t["bin2"], t["IF"] = v["bin1"], v["bin2"], v["IF"]
    return t


def _genome(g):
    return bytes(np.asarray(g["genome"], dtype=np.uint8)).decode().splitlines(keepends=True)


def _read_tables(path):
    from hichap_master_amd import coolio
    out = {}
    for grp in coolio.cooler_groups(path):
        with coolio.Cooler(f"{path}::{grp}") as c:
            cs = [(n, int(c.chromsizes[n])) for n in c.chromnames]
            b1, b2, cnt = c.pixels_table()
            w = c.weights() if "weight" in c._g("bins") else None
            out[int(grp)] = (cs, b1, b2, cnt, json.loads(c.info["metadata"]), w, c.chrom_offsets())
    return out


def _assert_table(got, want):
    cs, b1, b2, cnt = want
    assert got[0] == cs
    np.testing.assert_array_equal(got[1], b1)
    np.testing.assert_array_equal(got[2], b2)
    assert got[3].dtype == cnt.dtype
    np.testing.assert_array_equal(got[3], cnt)


def test_npz2cooler_tables_match_oracle_on_reference_libs(golden, tmp_path):
    from hichap_master_amd import matrixBuilding as mb
    g = golden("pairs_traditional")
    p = json.loads(str(g["params"]))
    W, L = _libs(g, p)
    gl = _genome(g)
    out = tmp_path / "S_Multi.cool"
    mb.NPZ2Cooler(W, str(out), gl, p["chroms"], onlyIntra=False, dtype="int")
    mb.NPZ2Cooler(L, str(out), gl, p["chroms"], onlyIntra=True, dtype="int")
    got = _read_tables(str(out))
    assert sorted(got) == sorted(p["wholeRes"] + p["localRes"])
    want = {**cooler_ref.npz2cooler_tables(W, gl, p["chroms"], False), **cooler_ref.npz2cooler_tables(L, gl, p["chroms"], True)}
    for res, t in want.items():
        _assert_table(got[res], t)
        assert got[res][4] == {"onlyIntra": str(res in p["localRes"])}
        # chromosome offsets = cooler's binnify (ceil(length / res))
        assert got[res][6][-1] == sum(-(-L_ // res) for _, L_ in t[0])
        assert t[1].size > 0 and np.all(t[1] <= t[2])
    # whole-genome groups hold trans pixels, local groups none
    for res in p["wholeRes"]:
        off = got[res][6]
        assert np.any(np.searchsorted(off, got[res][1], "right") != np.searchsorted(off, got[res][2], "right"))
    for res in p["localRes"]:
        off = got[res][6]
        np.testing.assert_array_equal(np.searchsorted(off, got[res][1], "right"),
                                      np.searchsorted(off, got[res][2], "right"))


def test_merge_sums_replicates(golden, tmp_path):
    from hichap_master_amd import matrixBuilding as mb
    g = golden("pairs_traditional")
    p = json.loads(str(g["params"]))
    W, L = _libs(g, p)
    gl = _genome(g)
    # replicate 2: every count doubled, a pixel dropped
    W2 = {res: {k: v.copy() for k, v in d.items()} for res, d in W.items()}
    for d in W2.values():
        for v in d.values():
            v["IF"] *= 2
    res0 = p["wholeRes"][0]
    W2[res0]["1"] = W2[res0]["1"][1:]
    f1, f2, fm = (str(tmp_path / n) for n in ("A_Multi.cool", "B_Multi.cool", "Merged_Multi.cool"))
    mb.NPZ2Cooler(W, f1, gl, p["chroms"], onlyIntra=False)
    mb.NPZ2Cooler(W2, f2, gl, p["chroms"], onlyIntra=False)
    for res in p["wholeRes"]:
        mb.merge_coolers(f"{fm}::{res}", [f"{f1}::{res}", f"{f2}::{res}"])
    got = _read_tables(fm)
    t1 = cooler_ref.npz2cooler_tables(W, gl, p["chroms"], False)
    t2 = cooler_ref.npz2cooler_tables(W2, gl, p["chroms"], False)
    for res in p["wholeRes"]:
        _assert_table(got[res], cooler_ref.merge_tables([t1[res], t2[res]]))


def test_intra_block_symmetrisation_follows_lil():
    """An intra block with lower entries: the upper cell takes its mirror's
    value (lil M[y, x] = M[x, y], then triu; NPZ2Cooler :290-293)."""
    from hichap_master_amd import matrixBuilding as mb
    rec = _rec({"bin1": np.array([0, 2, 1, 3, 4]), "bin2": np.array([2, 0, 1, 1, 4]),
                "IF": np.array([5.0, 7.0, 2.0, 4.0, 1.0])})
    gl = ["chr1\t500\n"]
    got = mb.npz2cooler_tables({100: {"1": rec}}, gl, ["#"], True, "float")[100]
    want = cooler_ref.npz2cooler_tables({100: {"1": rec}}, gl, ["#"], True, "float")[100]
    for a, b in zip(got[1:], want[1:]):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(got[3], [7.0, 2.0, 4.0, 1.0])


HAVE_H5 = all(os.path.exists(os.path.join("/opt/conda", q)) for q in ("include/hdf5.h", "lib/libhdf5.so"))


@pytest.mark.skipif(not HAVE_H5, reason="libhdf5 absent")
def test_constructed_cooler_read_by_libhdf5(golden, tmp_path):
    """The multi-resolution file NPZ2Cooler writes (then a weight column
    appended as balance_cooler does) is listed by libhdf5 exactly as h5.py
    lists it."""
    import shutil
    import subprocess
    from hichap_master_amd import h5, matrixBuilding as mb
    from tests.h5_listing import listing
    if shutil.which("gcc") is None:
        pytest.skip("gcc absent")
    g = golden("pairs_traditional")
    p = json.loads(str(g["params"]))
    W, L = _libs(g, p)
    gl = _genome(g)
    out = str(tmp_path / "S_Multi.cool")
    mb.NPZ2Cooler(W, out, gl, p["chroms"], onlyIntra=False)
    mb.NPZ2Cooler(L, out, gl, p["chroms"], onlyIntra=True)
    res = p["localRes"][0]
    n = int(_read_tables(out)[res][6][-1])
    h5.append_dataset(out, f"{res}/bins", "weight", np.linspace(0.5, 1.5, n),
                      {"tol": 1e-5, "min_nnz": 10, "cis_only": True, "ignore_diags": 1, "converged": True})
    exe = str(tmp_path / "make_h5_fixtures")
    subprocess.run(["gcc", "-O2", "-I/opt/conda/include", "-o", exe, os.path.join(GOLDEN, "make_h5_fixtures.c"),
                    "-L/opt/conda/lib", "-Wl,-rpath,/opt/conda/lib", "-lhdf5"], check=True)
    r = subprocess.run([exe, "dump", out], capture_output=True, text=True)
    assert r.returncode == 0 and not r.stderr, r.stderr[-2000:]
    assert sorted(r.stdout.splitlines()) == sorted(listing(out))


# ------------------------------------------------------------------ GPU
def _write_reps(tmp_path, text, n_reps=2):
    lines = text.splitlines(keepends=True)
    reps = []
    for k in range(n_reps):
        d = tmp_path / f"rep{k}"
        d.mkdir()
        part = lines[k::n_reps]
        half = len(part) // 2  # two files per replicate, `cat` together
        (d / f"S_R{k}_a_Valid.bed").write_bytes(b"".join(part[:half]))
        (d / f"S_R{k}_b_Valid.bed").write_bytes(b"".join(part[half:]))
        reps.append(str(d))
    return reps


@pytest.mark.gpu
def test_traditional_construction_end_to_end(golden, tmp_path):
    """Valid.bed text (two replicates) -> GPU binning -> replicate + merged
    multi-resolution coolers -> in-place ICE: tables equal the oracle's
    (oracle/pairs_ref binning + cooler_ref layout), weights equal the oracle
    ICE on the same tables (genome-wide / --cis-only), rtol 1e-9, the same
    iteration counts; attributes as cooler balance writes them."""
    from hichap_master_amd import _lib, coolio, matrixBuilding as mb
    from oracle import pairs_ref
    _lib.require_gpu()
    g = golden("pairs_traditional")
    p = json.loads(str(g["params"]))
    gl = _genome(g)
    gfile = tmp_path / "genome.txt"
    gfile.write_text("".join(gl))
    text = bytes(g["text"])
    reps = _write_reps(tmp_path, text)
    coolers = mb.TraditionalMatrixConstruction(str(tmp_path), reps, str(gfile), p["wholeRes"], p["localRes"],
                                               p["chroms"])
    assert [os.path.basename(c) for c in coolers] == ["S_R0_a_Multi.cool", "S_R1_a_Multi.cool", "Merged_Multi.cool"]
    rep_tabs = []
    for k, rep in enumerate(reps):
        txt = b"".join(open(os.path.join(rep, f), "rb").read() for f in sorted(os.listdir(rep)))
        Wo, Lo = pairs_ref.traditional_matrix_building(txt.decode().splitlines(keepends=True), gl, p["wholeRes"],
                                                       p["localRes"], p["chroms"])
        rep_tabs.append({**cooler_ref.npz2cooler_tables(Wo, gl, p["chroms"], False),
                         **cooler_ref.npz2cooler_tables(Lo, gl, p["chroms"], True)})
    merged = {res: cooler_ref.merge_tables([t[res] for t in rep_tabs]) for res in rep_tabs[0]}
    for path, want in zip(coolers, rep_tabs + [merged]):
        got = _read_tables(path)
        for res, t in want.items():
            _assert_table(got[res], t)
            cis = res in p["localRes"]
            cs, b1, b2, cnt = t
            wr, sr = ice_ref.balance(b1, b2, cnt.astype(np.int64), int(got[res][6][-1]), got[res][6], ignore_diags=1,
                                     cis_only=cis)
            np.testing.assert_allclose(got[res][5], wr, rtol=1e-9, equal_nan=True)
            with coolio.Cooler(f"{path}::{res}") as c:
                a = dict(c._g("bins")["weight"].attrs)
            assert bool(a["cis_only"]) == cis and int(a["ignore_diags"]) == 1


@pytest.mark.gpu
def test_haplotype_construction_end_to_end(golden, tmp_path):
    """The five allelic beds (one replicate, twice: two replicates) ->
    traditional / unimputed / imputed coolers + gap files per replicate and
    merged: the unimputed tables equal the oracle layout of the reference's
    own unimputed matrices (golden), the imputed cooler holds the two-step
    corrected matrices (oracle GenomeWideMatrixCorrection on the golden
    imputed matrix, rtol 1e-12), the merged unimputed counts are twice a
    replicate's, the traditional cooler is ICE-balanced in place."""
    from hichap_master_amd import _lib, matrixBuilding as mb
    from oracle import hichap_ref, pairs_ref
    from tests.test_impute_oracle import setup
    _lib.require_gpu()
    g = golden("impute_1res")
    p, _, UWd, _, IWd, _ = setup(g)
    gl = _genome(g)
    gfile = tmp_path / "genome.txt"
    gfile.write_text("".join(gl))
    reps = []
    for k in range(2):
        d = tmp_path / f"rep{k}"
        d.mkdir()
        for b in ("Bi_Allelic", "M_M", "P_P", "M_P", "P_M"):
            (d / f"S{k}_Valid_{b}.bed").write_bytes(bytes(g["text_" + b]))
        reps.append(str(d))
    out = mb.HaplotypeMatrixConstruction(str(tmp_path), reps, str(gfile), p["wholeRes"], p["localRes"],
                                         p["region"], p["min"], p["ratio"], p["chroms"])
    assert sorted(out) == ["Merged_", "S0_", "S1_"]
    genome = pairs_ref.load_genome(gl, p["chroms"])
    hap_lines = [f"{h}{c}\t{genome[c]}\n" for c in genome for h in "MP"]
    hap_chroms = [h + c for c in genome for h in "MP"]
    res = p["wholeRes"][0]
    hb, _ = pairs_ref.get_chro_bins_haplotypes(genome, res)
    UW = UWd[res]
    trad, unimp, imp = out["S0_"]
    got_u = _read_tables(unimp)
    want_u = cooler_ref.npz2cooler_tables({res: cooler_ref.whole_to_sparse_dict(hb, UW)}, hap_lines, hap_chroms, False)
    _assert_table(got_u[res], want_u[res])
    got_m = _read_tables(out["Merged_"][1])
    np.testing.assert_array_equal(got_m[res][3], 2 * got_u[res][3])
    # imputed: two-step genome-wide correction of the golden imputed matrix
    tb, _ = pairs_ref.get_chro_bins(genome, res)
    ds = mb.HaplotypeMatrixBuilding({b: os.path.join(reps[0], f"S0_Valid_{b}.bed") for b in
                                     ("Bi_Allelic", "M_M", "P_P", "M_P", "P_M")}, str(gfile), p["wholeRes"],
                                    p["localRes"], p["region"], p["min"], p["ratio"], p["chroms"])
    T = ds["Tradition_Whole"][res]["Matrix"]
    IW = IWd[res]
    Bal = hichap_ref.genome_wide_correction(tb, hb, T, IW)
    want_i = cooler_ref.npz2cooler_tables({res: cooler_ref.whole_to_sparse_dict(hb, Bal)}, hap_lines, hap_chroms,
                                          False, dtype="float")[res]
    got_i = _read_tables(imp)[res]
    np.testing.assert_array_equal(got_i[1], want_i[1])
    np.testing.assert_array_equal(got_i[2], want_i[2])
    np.testing.assert_allclose(got_i[3], want_i[3], rtol=1e-12, atol=0)
    assert got_i[3].dtype == np.float64
    assert _read_tables(trad)[res][5] is not None  # balanced in place
    gaps = np.load(os.path.join(tmp_path, "Cooler", "S0_Imputated_Gap.npz"), allow_pickle=True)  # our own file
    assert sorted(gaps.files) == [str(r) for r in sorted(p["localRes"])]
    # every localRes group of the imputed cooler: the oracle's
    # IntraChromMatrixCorrection (TwoStepCorrection per chromosome,
    # matrixBuilding.py:1026-1041, called at :1607-1614) of the imputed local
    # matrices, as NPZ2Cooler's float tables; the gap file's arrays are the
    # oracle's Gap_M / Gap_P (:1616-1617)
    got_all = _read_tables(imp)
    for lres in p["localRes"]:
        T_loc, I_loc = ds["Tradition_Local"][lres], ds["Imputated_Local"][lres]
        nor, gap_want = {}, {}
        for c in T_loc:
            nmm, npm, gm, gp = hichap_ref.two_step_correction(*(np.asarray(X, dtype=np.int64) for X in
                                                                 (T_loc[c], I_loc["M" + c], I_loc["P" + c])))
            nor["M" + c], nor["P" + c] = nmm, npm
            gap_want["M" + c], gap_want["P" + c] = gm, gp
        want_l = cooler_ref.npz2cooler_tables({lres: cooler_ref.intra_to_sparse_dict(nor)}, hap_lines, hap_chroms,
                                              True, dtype="float")[lres]
        got_l = got_all[lres]
        assert got_l[0] == want_l[0]
        np.testing.assert_array_equal(got_l[1], want_l[1])
        np.testing.assert_array_equal(got_l[2], want_l[2])
        assert got_l[3].dtype == np.float64
        np.testing.assert_allclose(got_l[3], want_l[3], rtol=1e-12, atol=0)
        gap_got = gaps[str(lres)].item()
        assert sorted(gap_got) == sorted(gap_want)
        for k in gap_want:
            np.testing.assert_array_equal(np.asarray(gap_got[k], dtype=np.int64), gap_want[k])
