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
