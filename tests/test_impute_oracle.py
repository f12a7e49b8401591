"""Imputation oracle (oracle/impute_ref.py) against the reference's own
imputation statements (tests/golden/impute_*.npz) — no GPU."""
import json

import numpy as np
import pytest

from oracle import impute_ref, pairs_ref

CASES = ["impute_1res", "impute_fine"]


def lines(a):
    return bytes(np.asarray(a, dtype=np.uint8)).decode().splitlines(keepends=True)


def dense_lib(g, prefix, shapes):
    out = {}
    for k in g:
        if k.startswith(prefix + "/") and k.endswith("/bin1"):
            _, res, key, _ = k.split("/")
            M = np.zeros(shapes[(int(res), key)], dtype=np.int64)
            base = f"{prefix}/{res}/{key}/"
            M[g[base + "bin1"], g[base + "bin2"]] = g[base + "IF"].astype(np.int64)
            out.setdefault(int(res), {})[key] = M
    return out


def shapes_of(genome, p):
    sh = {}
    for res in p["wholeRes"]:
        sh[(res, "__whole__")] = (pairs_ref.get_chro_bins_haplotypes(genome, res)[1],) * 2
    for res in p["localRes"]:
        for h in "MP":
            for c, l in genome.items():
                sh[(res, h + c)] = (l // res + 1,) * 2
    return sh


def setup(g):
    p = json.loads(str(g["params"]))
    genome = pairs_ref.load_genome(lines(g["genome"]), p["chroms"])
    sh = shapes_of(genome, p)
    UW = {r: d["__whole__"] for r, d in dense_lib(g, "uwhole", sh).items()}
    UL = dense_lib(g, "ulocal", sh)
    for res in p["localRes"]:
        UL.setdefault(res, {})
        for key in [k for (r, k) in sh if r == res]:
            UL[res].setdefault(key, np.zeros(sh[(res, key)], dtype=np.int64))
    IW = {r: d["__whole__"] for r, d in dense_lib(g, "iwhole", sh).items()}
    IL = dense_lib(g, "ilocal", sh)
    return p, genome, UW, UL, IW, IL


@pytest.mark.parametrize("case", CASES)
def test_impute_oracle_matches_reference(golden, case):
    g = golden(case)
    p, genome, UW, UL, IW, IL = setup(g)
    src = {k: lines(g["text_" + k]) for k in ("M_M", "P_P")}
    W, L = impute_ref.impute(src, genome, p["chroms"], p["wholeRes"], p["localRes"], p["region"], p["min"],
                             p["ratio"], UW, UL)
    for res in p["wholeRes"]:
        np.testing.assert_array_equal(W[res], IW[res])
        assert (IW[res] != UW[res]).any()
    for res in p["localRes"]:
        for key, M in L[res].items():
            np.testing.assert_array_equal(M, IL[res].get(key, np.zeros_like(M)), err_msg=key)


def test_unimputed_golden_matches_pairs_oracle(golden):
    g = golden("impute_1res")
    p, genome, UW, UL, IW, IL = setup(g)
    src = {k: lines(g["text_" + k]) for k in ("M_M", "P_P", "M_P", "P_M")}
    whole, local = pairs_ref.haplotype_counts(src, genome, p["chroms"], p["wholeRes"], p["localRes"])
    res = p["wholeRes"][0]
    b1, b2, c = pairs_ref.counter_to_pixels(whole[res])
    M = np.zeros_like(UW[res])
    M[b1, b2] = c
    M[b2, b1] = c
    np.testing.assert_array_equal(M, UW[res])


def test_stale_window_missing_raises():
    genome = {"1": 5_000_000, "2": 5_000_000}
    UW = {500000: np.ones((44, 44), dtype=np.int64)}  # M1 M2 P1 P2, 11 bins each
    src = {"M_M": [], "P_P": ["chr1\t2000000\tchr2\t2500000\tR1\n"]}
    with pytest.raises(NameError):
        impute_ref.impute(src, genome, ["#"], [500000], [], 1_000_000, 2, 0.9, UW, {})
