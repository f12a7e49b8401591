"""Pair-binning oracle (oracle/pairs_ref.py) against golden vectors produced by
the reference's own TraditionalMatrixBuilding / TraditionalMatrixInAllelic /
HaplotypeMatrixBuilding passes (tests/golden/make_golden_pairs.py)."""
import json

import numpy as np
import pytest

from oracle import pairs_ref


def _text(a):
    return bytes(np.asarray(a, dtype=np.uint8)).decode()


def _lines(a):
    return _text(a).splitlines(keepends=True)


def _golden_keys(g, prefix):
    out = {}
    for k in g:
        if k.startswith(prefix + "/"):
            _, res, key, f = k.split("/")
            out.setdefault((int(res), key), {})[f] = g[k]
    return out


@pytest.mark.parametrize("case", ["pairs_traditional", "pairs_traditional_allchroms"])
def test_traditional_sparse_dicts(golden, case):
    g = golden(case)
    p = json.loads(str(g["params"]))
    W, L = pairs_ref.traditional_matrix_building(_lines(g["text"]), _lines(g["genome"]),
                                                 p["wholeRes"], p["localRes"], p["chroms"])
    for prefix, lib in (("whole", W), ("local", L)):
        gk = _golden_keys(g, prefix)
        got = {(res, key): arr for res, d in lib.items() for key, arr in d.items()}
        assert set(got) == set(gk)
        for k, arr in got.items():
            for f in ("bin1", "bin2", "IF"):
                np.testing.assert_array_equal(arr[f], gk[k][f], err_msg=f"{k} {f}")


def _check_dense(gk, whole, local):
    for (res, key), d in gk.items():
        counter = whole[res] if key == "__whole__" else local[res][key]
        b1, b2, c = pairs_ref.counter_to_pixels(counter)
        np.testing.assert_array_equal(b1, d["bin1"])
        np.testing.assert_array_equal(b2, d["bin2"])
        np.testing.assert_array_equal(c.astype(np.float64), d["IF"])


def test_allelic_traditional_dense(golden):
    g = golden("pairs_allelic_traditional")
    p = json.loads(str(g["params"]))
    genome = pairs_ref.load_genome(_lines(g["genome"]), p["chroms"])
    whole, local = pairs_ref.traditional_counts(_lines(g["text"]), genome, p["chroms"], p["wholeRes"],
                                                p["localRes"], cols=(0, 1, 2, 3))
    gk = _golden_keys(g, "whole")
    gk.update(_golden_keys(g, "local"))
    assert sum(1 for k in gk if k[1] != "__whole__") == len(genome)
    _check_dense(gk, whole, local)


def test_haplotype_unimputed_dense(golden):
    g = golden("pairs_haplotype_unimputed")
    p = json.loads(str(g["params"]))
    genome = pairs_ref.load_genome(_lines(g["genome"]), p["chroms"])
    src = {k: _lines(g["text_" + k]) for k in ("M_M", "P_P", "M_P", "P_M")}
    whole, local = pairs_ref.haplotype_counts(src, genome, p["chroms"], p["wholeRes"], p["localRes"])
    gk = _golden_keys(g, "whole")
    gk.update(_golden_keys(g, "local"))
    assert sum(1 for k in gk if k[1] != "__whole__") == 2 * len(genome)
    _check_dense(gk, whole, local)


def test_oracle_raises_like_reference():
    genome = {"1": 1_000_000, "2": 500_000}
    ok = "r chr1 + 5 0 0 100 0 chr2 - 5 0 0 200 0\n"
    w, _ = pairs_ref.traditional_counts([ok], genome, ["#"], [100000], [])
    assert sum(w[100000].values()) == 1
    with pytest.raises(IndexError):   # too few fields
        pairs_ref.traditional_counts(["r chr1 + 5 0 0 100 0 chr2\n"], genome, ["#"], [100000], [])
    with pytest.raises(ValueError):   # non-integer position
        pairs_ref.traditional_counts([ok.replace(" 100 ", " 1e2 ")], genome, ["#"], [100000], [])
    with pytest.raises(KeyError):     # passes '#' but not in the genome
        pairs_ref.traditional_counts([ok.replace("chr2", "chr3")], genome, ["#"], [100000], [])
    # filtered out by the chroms check: skipped, no error
    w, _ = pairs_ref.traditional_counts([ok.replace("chr2", "chrY")], genome, ["#"], [100000], [])
    assert sum(w[100000].values()) == 0
    with pytest.raises(IndexError):   # bin past the end of the whole matrix
        pairs_ref.traditional_counts([ok.replace(" 200 ", " 900000 ")], genome, ["#"], [100000], [])
