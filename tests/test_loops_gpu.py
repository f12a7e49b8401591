"""HICCUPS on the GPU (hh_hiccups_* through the C-ABI) against the reference's
golden calls and the CPU oracle.  Raw reads are integer sums (exact); the
balanced / expected neighbourhood sums come from prefix differences, so
they are compared at rtol 1e-10 (call sets must be identical)."""
import numpy as np
import pytest

from oracle import loops_ref

pytestmark = pytest.mark.gpu

CASES = ["loops_trad_n360", "loops_allelic_n300"]


@pytest.fixture(scope="module")
def lp():
    from hichap_master_amd import _lib, loops
    _lib.require_gpu()
    return loops


def _args(g):
    allelic = bool(g["allelic"])
    return g["H"], g["weights"], int(g["res"]), allelic, (list(g["gaps"]) if allelic else None)


def _flat(D):
    keys = sorted(D)
    return np.array(keys, dtype=np.int64).reshape(-1, 2), np.array([D[k] for k in keys]).reshape(-1, 4)


@pytest.mark.parametrize("case", CASES)
def test_pcaller_matches_reference(lp, golden, case):
    g = golden(case)
    D, L = lp.pcaller(*_args(g))
    pd, vd = _flat(D)
    pl, vl = _flat(L)
    np.testing.assert_array_equal(pd, g["pos"])
    np.testing.assert_array_equal(pl, g["pos"])
    np.testing.assert_allclose(vd, g["donut"], rtol=1e-9)
    np.testing.assert_allclose(vl, g["ll"], rtol=1e-9)


def _synthetic(seed, N, res, depth=40.0):
    rng = np.random.default_rng(seed)
    i = np.arange(N)
    d = np.abs(i[:, None] - i[None, :])
    lam = depth * (d + 1.0) ** -1.05 * rng.lognormal(0, 0.2, N)[:, None]
    lam = np.triu(lam) + np.triu(lam, 1).T
    for _ in range(N // 25):
        a = int(rng.integers(5, N - 80))
        b = a + int(rng.integers(6, 60))
        lam[a - 1:a + 2, b - 1:b + 2] *= 4.0
    H = rng.poisson(np.triu(lam))
    H = np.triu(H) + np.triu(H, 1).T
    gaps = rng.choice(N, size=N // 80, replace=False)
    H[gaps, :] = 0
    H[:, gaps] = 0
    rs = H.sum(1).astype(float)
    w = np.where(rs > 0, 1.0 / np.sqrt(np.maximum(rs, 1.0)), np.nan)
    return H.astype(np.int64), w, np.sort(gaps)


@pytest.mark.parametrize("res,allelic", [(20000, False), (10000, False), (20000, True)])
def test_neighbourhood_sums_vs_oracle(lp, res, allelic):
    H, w, gaps = _synthetic(5 + res // 10000, 700, res)
    P = loops_ref.prepare(H, w, res, allelic)
    xi, yi = loops_ref.candidates(P, list(gaps))
    So, Eo, vo, wo = loops_ref.neighbourhood(P, xi, yi)
    B = lp.bands(H, w, res, allelic)
    nb = lp.Neighbourhood(B)
    S, E, valid, widths = nb.run(xi, yi)
    nb.close()
    assert [(a, b) for a, b, _ in widths] == [(a, b) for a, b, _ in wo]
    np.testing.assert_array_equal(valid, vo)
    for fl in "KY":
        np.testing.assert_allclose(S[fl], So[fl], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(E[fl], Eo[fl], rtol=1e-10, atol=1e-12)
    Do, Lo = loops_ref.significance(P, xi, yi, So, Eo, vo)
    D, L = lp.significance(B, xi, yi, S, E, valid)
    assert sorted(D) == sorted(Do) and len(D) > 0
    for k in D:
        np.testing.assert_allclose(D[k], Do[k], rtol=1e-9)
        np.testing.assert_allclose(L[k], Lo[k], rtol=1e-9)


def test_no_candidates(lp):
    H = np.zeros((200, 200), dtype=np.int64)
    D, L = lp.pcaller(H, np.ones(200), 40000, allelic=True, gap=[])
    assert D == {} and L == {}


def test_low_coverage_band_calls_nothing(lp):
    """Every expected value below 2**(-2/3): the reference's lambdachunk has no
    chunk, p = q = 1 and nothing is called (this used to raise)."""
    rng = np.random.default_rng(12)
    N = 300
    up = np.triu(rng.poisson(0.04, size=(N, N)), 1)
    H = (up + up.T).astype(np.int64)
    B = lp.bands(H, np.ones(N), 40000)
    xi, yi = lp.candidates(B)
    assert xi.size > 0
    D, L = lp.pcaller(H, np.ones(N), 40000)
    assert D == {} and L == {}


def test_call_peaks_writes_reference_format(lp, golden, tmp_path):
    g = golden("loops_trad_n360")
    out = tmp_path / "loops.txt"
    res = lp.call_peaks({"chr1": (g["H"], g["weights"])}, int(g["res"]), str(out))
    lines = out.read_text().splitlines()
    assert lines[0].split("\t")[0] == "chromLabel" and len(lines) == 1 + len(g["pos"])
    first = lines[1].split("\t")
    assert first[0] == "chr1" and int(first[1]) == g["pos"][0][0] and int(first[2]) == g["pos"][0][1]
    assert len(res["chr1"][0]) == len(g["pos"])
