"""HICCUPS: oracle (oracle/loops_ref.py) against the reference's own pcaller
(tests/golden/loops_*.npz), and the host glue of hichap_master_amd.loops
(vectorised candidates / BH / lambda chunks) against the oracle — no GPU."""
import numpy as np
import pytest

from hichap_master_amd import loops
from oracle import loops_ref

CASES = ["loops_trad_n360", "loops_allelic_n300"]


def _args(g):
    allelic = bool(g["allelic"])
    return g["H"], g["weights"], int(g["res"]), allelic, (list(g["gaps"]) if allelic else None)


def _flat(D):
    keys = sorted(D)
    return np.array(keys, dtype=np.int64).reshape(-1, 2), np.array([D[k] for k in keys]).reshape(-1, 4)


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference(golden, case):
    g = golden(case)
    D, L = loops_ref.pcaller(*_args(g))
    pd, vd = _flat(D)
    pl, vl = _flat(L)
    np.testing.assert_array_equal(pd, g["pos"])
    np.testing.assert_array_equal(pl, g["pos"])
    np.testing.assert_allclose(vd, g["donut"], rtol=1e-12)
    np.testing.assert_allclose(vl, g["ll"], rtol=1e-12)
    assert len(pd) > 0


@pytest.mark.parametrize("case", CASES)
def test_host_bands_and_candidates_match_oracle(golden, case):
    H, w, res, allelic, gap = _args(golden(case))
    P = loops_ref.prepare(H, w, res, allelic)
    B = loops.bands(H, w, res, allelic)
    np.testing.assert_array_equal(B["Hb"], P["Hb"])
    np.testing.assert_array_equal(B["Cb"], P["Cb"])
    np.testing.assert_array_equal(B["Eall"], P["Eall"])
    xo, yo = loops_ref.candidates(P, gap)
    xg, yg = loops.candidates(B, gap)
    np.testing.assert_array_equal(np.sort(xo * 100000 + yo), np.sort(xg * 100000 + yg))


def test_bh_by_value_equals_statsmodels_restatement():
    rng = np.random.default_rng(3)
    for n in (1, 2, 7, 500):
        p = rng.choice(rng.random(max(1, n // 3)), size=n)  # many ties
        np.testing.assert_array_equal(loops._bh_by_value(p), loops_ref.fdr_bh(p))


def test_lambda_chunks_edges_match():
    E = np.array([0.3, 1.0, 1.26, 2 ** (1 / 3.), 5.0, 17.2])
    pool = loops_ref.lambdachunk(E)
    assert [(lv, rv) for lv, rv, _ in pool] == loops.lambda_chunks(E)


def test_significance_host_equals_oracle(golden):
    """The vectorised significance stage on the oracle's neighbourhood sums."""
    g = golden("loops_trad_n360")
    H, w, res, allelic, gap = _args(g)
    P = loops_ref.prepare(H, w, res, allelic)
    xi, yi = loops_ref.candidates(P, gap)
    S, E, valid, _ = loops_ref.neighbourhood(P, xi, yi)
    B = loops.bands(H, w, res, allelic)
    D, L = loops.significance(B, xi, yi, S, E, valid)
    pd, vd = _flat(D)
    np.testing.assert_array_equal(pd, g["pos"])
    np.testing.assert_array_equal(vd, g["donut"])
