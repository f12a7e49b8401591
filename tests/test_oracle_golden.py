"""The CPU oracle against golden vectors produced by the reference's own
functions (tests/golden/make_golden.py)."""
import numpy as np
import pytest

from oracle import hichap_ref, structure_ref

TWOSTEP = ["twostep_gaps_n96", "twostep_gaps_n160", "twostep_nogapM_n80"]


@pytest.mark.parametrize("name", TWOSTEP)
def test_twostep_oracle(golden, name):
    g = golden(name)
    nmm, npm, gm, gp = hichap_ref.two_step_correction(g["TM"], g["MM"], g["PM"])
    np.testing.assert_array_equal(gm, g["Gap_M"])
    np.testing.assert_array_equal(gp, g["Gap_P"])
    np.testing.assert_allclose(nmm, g["Nor_MM"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(npm, g["Nor_PM"], rtol=1e-12, atol=0)


def test_genomewide_oracle(golden):
    g = golden("genomewide_3chrom")
    names = [str(x) for x in g["names"]]
    sizes = [int(x) for x in g["sizes"]]
    n = sum(sizes)
    bins, hbins, s = {}, {}, 0
    for nm, L in zip(names, sizes):
        bins[nm] = (s, s + L - 1)
        hbins["M" + nm] = (s, s + L - 1)
        hbins["P" + nm] = (n + s, n + s + L - 1)
        s += L
    out = hichap_ref.genome_wide_correction(bins, hbins, g["T_M"], g["H_M"])
    np.testing.assert_allclose(out, g["Nor"], rtol=1e-12, atol=0)


@pytest.mark.parametrize("name", ["compartment_n150", "compartment_n260"])
def test_compartment_oracle(golden, name):
    g = golden(name)
    dec, G, NG = structure_ref.distance_decay(g["M"])
    np.testing.assert_array_equal(G, g["G"])
    np.testing.assert_array_equal(NG, g["NG"])
    np.testing.assert_allclose(dec, g["decline"], rtol=1e-12, atol=0)
    pcs, C, OE = structure_ref.get_pca(dec, g["M"], NG)
    np.testing.assert_allclose(OE, g["OE"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(C, g["Cor"], rtol=0, atol=1e-12)
    # PCA sign convention is solver dependent: compare up to sign
    for k in range(3):
        s = np.sign(np.dot(pcs[k], g["pcs"][k]))
        np.testing.assert_allclose(s * pcs[k], g["pcs"][k], atol=1e-9)
    pc, _ = structure_ref.select_pc(C, OE[NG], pcs)
    full = np.zeros(g["M"].shape[0])
    full[NG] = pc
    np.testing.assert_allclose(full, g["pc"], atol=1e-9)
    np.testing.assert_array_equal(np.sign(full), np.sign(g["pc"]))
    raw = np.zeros((3, g["M"].shape[0]))
    raw[:, NG] = pcs
    sel, _ = structure_ref.select_allelic_pc(raw, g["trad"])
    s = np.sign(np.dot(sel, g["allelic"]))
    np.testing.assert_allclose(s * sel, g["allelic"], atol=1e-9)


@pytest.mark.parametrize("name,test", [("di_ttest_n220", "ttest"), ("di_chitest_n220", "chitest")])
def test_di_oracle(golden, name, test):
    g = golden(name)
    gap = structure_ref.get_gap(g["M"], int(g["lb"]) * 40000, 40000)
    np.testing.assert_array_equal(gap, g["gap"])
    di = structure_ref.get_di(g["M"], gap, int(g["window_bins"]), test)
    np.testing.assert_allclose(di, g["DI"], rtol=1e-12, atol=1e-300)


def _sliding_loop(M, dec, step):
    """Literal restatement of Sliding_Approach's double loop (:285-297)."""
    N = M.shape[0]
    out = np.zeros(M.shape)
    for i in range(N):
        for j in range(N):
            if i < step or j < step or i > N - step - 1 or j > N - step - 1:
                out[i][j] = M[i][j] / dec[abs(i - j)]
            else:
                o = M[i - step:i + step + 1, j - step:j + step + 1].sum()
                e = (3 * dec[abs(i - j)] + 2 * dec[abs(i - j - 1)] + 2 * dec[abs(i - j + 1)] + dec[abs(i - j - 2)]
                     + dec[abs(i - j + 2)])
                out[i][j] = o / e
    return out


@pytest.mark.parametrize("N,step", [(30, 2), (9, 4), (7, 4), (25, 1)])
def test_sliding_oe_vectorised_equals_loop(N, step):
    rng = np.random.default_rng(N + step)
    M = rng.poisson(3.0, size=(N, N)).astype(np.float64) + rng.random((N, N))
    M = M + M.T
    dec = rng.random(N) + 0.5
    np.testing.assert_allclose(structure_ref.sliding_oe(M, dec, step), _sliding_loop(M, dec, step), rtol=1e-13)
    with pytest.raises(IndexError):
        structure_ref.sliding_oe(M, dec, 0)


@pytest.mark.parametrize("name", ["compartment_sa_n120", "compartment_sa_n150"])
def test_compartment_sliding_approach_oracle(golden, name):
    """Get_PCA(SA=True) golden (make_golden.py main_sa, the reference run)."""
    g = golden(name)
    pcs, C, OE = structure_ref.get_pca(g["decline"], g["M"], g["NG"], SA=True, res=int(g["res"]))
    np.testing.assert_allclose(OE, g["OE"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(C, g["Cor"], rtol=0, atol=1e-12)
    for k in range(3):
        s = np.sign(np.dot(pcs[k], g["pcs"][k]))
        np.testing.assert_allclose(s * pcs[k], g["pcs"][k], atol=1e-9)
    pc, _ = structure_ref.select_pc(C, OE[g["NG"]], pcs)
    np.testing.assert_allclose(pc, g["pc"][g["NG"]], atol=1e-9)
