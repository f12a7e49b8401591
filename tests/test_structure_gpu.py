"""Compartment (decay, O/E, Pearson on fp64 MFMA, top-3 PCA, PC selection)
and DI TAD scan on the GPU vs the reference's golden outputs and the oracle."""
import numpy as np
import pytest

from hichap_master_amd import synth
from oracle import structure_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def SF():
    from hichap_master_amd import _lib
    from hichap_master_amd.StructureFind import StructureFind
    _lib.require_gpu()
    return StructureFind


def _match_sign(a, b):
    return a * np.sign(np.dot(a, b))


@pytest.mark.parametrize("name", ["compartment_n150", "compartment_n260"])
def test_compartment_matches_reference_golden(SF, golden, name):
    g = golden(name)
    sf = SF(Res=100000)
    M = g["M"]
    dec, G, NG = sf.Distance_Decay(M=M, G_array=None)
    np.testing.assert_array_equal(G, g["G"])
    np.testing.assert_array_equal(NG, g["NG"])
    np.testing.assert_allclose(dec, g["decline"], rtol=1e-12, atol=0)
    pcs, Cor, OE = sf.Get_PCA(distance_bin=dec.copy(), M=M, NG_array=NG)
    np.testing.assert_allclose(np.asarray(Cor), g["Cor"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(np.asarray(OE), g["OE"], rtol=1e-12, atol=0)
    for k in range(3):
        np.testing.assert_allclose(_match_sign(pcs[k], g["pcs"][k]), g["pcs"][k], atol=1e-9)
    pc = sf.Select_PC_new(Cor, OE[NG], pcs)
    full = np.zeros(M.shape[0])
    full[NG] = pc
    np.testing.assert_allclose(full, g["pc"], atol=1e-9)
    np.testing.assert_array_equal(np.sign(full), np.sign(g["pc"]))
    # the whole per-chromosome body in one call
    np.testing.assert_allclose(SF(Res=100000).compartment(M), g["pc"], atol=1e-9)
    # haplotype selection (sign = solver convention: compare up to sign)
    al = SF(Res=100000).compartment(M, Tranditional_PC=g["trad"])
    np.testing.assert_allclose(_match_sign(al, g["allelic"]), g["allelic"], atol=1e-9)


def test_select_pc_on_host_arrays(SF, golden):
    g = golden("compartment_n150")
    sf = SF(Res=100000)
    NG = g["NG"]
    pc = sf.Select_PC_new(g["Cor"], g["OE"][NG], g["pcs"])
    ref, _ = structure_ref.select_pc(g["Cor"], g["OE"][NG], g["pcs"])
    np.testing.assert_array_equal(pc, ref)


@pytest.mark.parametrize("N", [700, 1500])
def test_compartment_vs_oracle_larger(SF, N):
    rng = np.random.default_rng(N)
    M = synth.dense_chrom(N, rng, A=80.0, comp_len=(20, 60), gap_frac=0.03).astype(np.float64)
    sf = SF(Res=25000)
    dec, G, NG = sf.Distance_Decay(M=M, G_array=None)
    d_ref, G_ref, NG_ref = structure_ref.distance_decay(M)
    np.testing.assert_array_equal(NG, NG_ref)
    np.testing.assert_allclose(dec, d_ref, rtol=1e-12)
    pcs, Cor, OE = sf.Get_PCA(distance_bin=dec.copy(), M=M, NG_array=NG)
    p_ref, C_ref, _ = structure_ref.get_pca(d_ref, M, NG_ref)
    C = np.asarray(Cor)
    np.testing.assert_allclose(C, C_ref, atol=1e-11)
    np.testing.assert_allclose(C, C.T, atol=1e-15)  # corrcoef divides rows then columns: not bitwise symmetric
    # PC1 always well separated; PC2/3 compared through the selected vector
    np.testing.assert_allclose(_match_sign(pcs[0], p_ref[0]), p_ref[0], atol=1e-8)
    full = sf.compartment(M)
    ref_full, _, _, _ = structure_ref.compartment(M)
    big = np.abs(ref_full) > 1e-6
    np.testing.assert_array_equal(np.sign(full[big]), np.sign(ref_full[big]))
    np.testing.assert_allclose(full, ref_full, atol=1e-7)


@pytest.mark.parametrize("name,test", [("di_ttest_n220", "ttest"), ("di_chitest_n220", "chitest")])
def test_di_matches_reference_golden(SF, golden, name, test):
    g = golden(name)
    sf = SF(Res=40000)
    sf.TAD_parameter_init(200000, 4000000, 3, 600000, test)
    gap, di = sf.di_scan(g["M"])
    np.testing.assert_array_equal(gap, g["gap"])
    np.testing.assert_allclose(di, g["DI"], rtol=1e-12, atol=1e-300)
    np.testing.assert_array_equal(np.sign(di), np.sign(g["DI"]))
    assert sf.Gap_Filter(gap, g["M"]) == list(g["gap_filtered"])


def test_di_large_vs_oracle(SF):
    rng = np.random.default_rng(9)
    N = 3000
    M = synth.dense_chrom(N, rng, A=30.0, gap_frac=0.03).astype(np.float64)
    sf = SF(Res=10000)
    sf.TAD_parameter_init(50000, 4000000, 3, 600000, "ttest")
    gap, di = sf.di_scan(M)
    gref = structure_ref.get_gap(M, 50000, 10000)
    np.testing.assert_array_equal(gap, gref)
    dref = structure_ref.get_di(M, gref, 60, "ttest")
    np.testing.assert_allclose(di, dref, rtol=1e-11, atol=1e-300)


def test_compartment_device_tensor_input(SF):
    """A device-resident torch tensor goes to the C-ABI without a host copy
    and gives the same PC as the NumPy input."""
    import torch
    rng = np.random.default_rng(3)
    M = synth.dense_chrom(600, rng, A=30.0, gap_frac=0.03).astype(np.float64)
    a = SF(Res=100000).compartment(M)
    b = SF(Res=100000).compartment(torch.from_numpy(M).cuda())
    np.testing.assert_array_equal(a, b)


def _balanced_dense(b1, b2, c, w, lo, N):
    """cooler.matrix(balance=True).fetch(chrom) + np.nan_to_num (Data_preprocess
    :853-854) in NumPy: count * w[bin1] * w[bin2], symmetric."""
    sel = (b1 >= lo) & (b1 < lo + N) & (b2 >= lo) & (b2 < lo + N)
    i, j = b1[sel] - lo, b2[sel] - lo
    v = c[sel].astype(np.float64)
    if w is not None:
        v = v * w[b1[sel]] * w[b2[sel]]
    M = np.zeros((N, N))
    M[i, j] = v
    M[j, i] = v
    return np.nan_to_num(M)


@pytest.mark.parametrize("balanced,test", [(True, "ttest"), (True, "chitest"), (False, "ttest")])
def test_tad_scan_from_pixels(SF, balanced, test):
    """di_scan_pixels (device band from the pixel table + ICE weights) equals
    di_scan on the dense balanced matrix bitwise, and the oracle."""
    from hichap_master_amd import ice
    from hichap_master_amd._lib import call, ptr
    from hichap_master_amd.StructureFind import column_band
    rng = np.random.default_rng(31)
    b1, b2, c, off = synth.coo_genome([900, 1200], rng, A=30.0, trans_density=0.01)
    n = int(off[-1])
    w = ice.balance(b1, b2, c, n, off, max_iters=300)[0] if balanced else None
    sf = SF(Res=10000)
    sf.TAD_parameter_init(50000, 4000000, 3, 300000, test)
    for k in range(2):
        lo, N = int(off[k]), int(off[k + 1] - off[k])
        M = _balanced_dense(b1, b2, c, w, lo, N)
        gap, di = sf.di_scan_pixels(b1, b2, c, w, lo, N)
        gd, dd = sf.di_scan(M)
        np.testing.assert_array_equal(gap, gd)
        np.testing.assert_array_equal(di, dd)
        gref = list(structure_ref.get_gap(M, 50000, 10000))
        gref = sorted(set(gref) | {0, N - 1})
        np.testing.assert_array_equal(gap, gref)
        dref = structure_ref.get_di(M, np.array(gref), 30, test)
        # a DI near 0 is a difference of near-equal up / down sums: its
        # rounding error scales with the scan's magnitudes, not with itself
        np.testing.assert_allclose(di, dref, rtol=1e-11, atol=1e-13 * np.abs(dref).max())
        # the band itself, host mode
        B = 30
        band = np.empty((2 * B + 1, N))
        cf = np.ascontiguousarray(c, dtype=np.float64)
        call("hh_band_from_pixels", ptr(b1), ptr(b2), ptr(cf), b1.size,
             None if w is None else ptr(w), 0 if w is None else n, lo, N, B, ptr(band), 0, None)
        np.testing.assert_array_equal(band, column_band(M, B))


def test_tad_scan_from_pixels_empty(SF):
    sf = SF(Res=10000)
    sf.TAD_parameter_init(50000, 4000000, 3, 300000, "ttest")
    e = np.zeros(0, np.int64)
    gap, di = sf.di_scan_pixels(e, e, np.zeros(0), None, 0, 200)
    np.testing.assert_array_equal(gap, np.arange(200))
    assert not di.any()


@pytest.mark.parametrize("name", ["compartment_sa_n120", "compartment_sa_n150"])
def test_sliding_approach_matches_reference_golden(SF, golden, name):
    """Get_PCA(SA=True): Sliding_Approach O/E (StructureFind.py:274-299) on the
    device, against the reference's own output."""
    g = golden(name)
    sf = SF(Res=int(g["res"]))
    M = g["M"]
    dec, G, NG = sf.Distance_Decay(M=M, G_array=None)
    np.testing.assert_array_equal(NG, g["NG"])
    pcs, Cor, OE = sf.Get_PCA(distance_bin=dec.copy(), M=M, NG_array=NG, SA=True)
    np.testing.assert_allclose(np.asarray(OE), g["OE"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(np.asarray(Cor), g["Cor"], rtol=0, atol=1e-12)
    for k in range(3):
        np.testing.assert_allclose(_match_sign(pcs[k], g["pcs"][k]), g["pcs"][k], atol=1e-9)
    pc = sf.Select_PC_new(Cor, OE[NG], pcs)
    np.testing.assert_allclose(pc, g["pc"][NG], atol=1e-9)
    np.testing.assert_array_equal(np.sign(pc), np.sign(g["pc"][NG]))
    # the same matrix object back on the plain O/E
    dec2, _, NG2 = sf.Distance_Decay(M=M, G_array=None)
    _, Cor2, OE2 = sf.Get_PCA(distance_bin=dec2.copy(), M=M, NG_array=NG2)
    ref = structure_ref.get_pca(dec2, M, NG2)
    np.testing.assert_allclose(np.asarray(OE2), ref[2], rtol=1e-12)


def test_sliding_approach_vs_oracle_larger_and_errors(SF):
    rng = np.random.default_rng(5)
    M = synth.dense_chrom(900, rng, A=80.0, comp_len=(20, 60), gap_frac=0.03).astype(np.float64)
    sf = SF(Res=20000)  # step 15
    dec, G, NG = sf.Distance_Decay(M=M, G_array=None)
    pcs, Cor, OE = sf.Get_PCA(distance_bin=dec.copy(), M=M, NG_array=NG, SA=True)
    p_ref, C_ref, OE_ref = structure_ref.get_pca(dec, M, NG, SA=True, res=20000)
    np.testing.assert_allclose(np.asarray(OE), OE_ref, rtol=1e-12)
    np.testing.assert_allclose(np.asarray(Cor), C_ref, atol=1e-11)
    np.testing.assert_allclose(_match_sign(pcs[0], p_ref[0]), p_ref[0], atol=1e-8)
    with pytest.raises(IndexError):
        SF(Res=400000).Get_PCA(distance_bin=dec.copy(), M=M, NG_array=NG, SA=True)


def test_compartment_keeps_refilled_cor_and_oe(SF, golden):
    """Compartment() fills Cor_Martrix_Dict / OE_Matrix_Dict with the
    gap-refilled matrices (StructureFind.py:550-554) that Plot_Compartment
    reads: against the reference's golden Cor / O/E through the reference's
    Refill_Gap loops (oracle)."""
    g = golden("compartment_n150")
    M = g["M"]
    sf = SF(Res=100000)
    sf.Compartment(Matrix_Dict={"chr1": M})
    NG = g["NG"]
    np.testing.assert_allclose(sf.Cor_Martrix_Dict["chr1"], structure_ref.refill_gap(M, g["Cor"], NG, "Cor"),
                               rtol=0, atol=1e-12)
    np.testing.assert_allclose(sf.OE_Matrix_Dict["chr1"], structure_ref.refill_gap(M, g["OE"], NG, "OE"),
                               rtol=1e-12, atol=0)
    assert list(sf.Cor_Martrix_Dict) == ["chr1"] and "chr1" in sf.OE_Matrix_Dict


def test_compartment_frees_device_state_and_sa_thunks(SF, golden):
    """Compartment() keeps no chromosome's hh_comp alive (the
    refilled-matrix thunks are built from host inputs), and with SA=True the
    refilled O/E and Cor equal Refill_Gap of Get_PCA's own SA outputs."""
    g = golden("compartment_sa_n150")
    M = g["M"]
    res = int(g["res"]) if "res" in g else 20000
    sf = SF(Res=res)
    sf.Compartment(SA=True, Matrix_Dict={"chrA": M, "chrB": M[:120, :120].copy()})
    assert sf._comp is None
    for name, X in (("chrA", M), ("chrB", M[:120, :120])):
        ref = SF(Res=res)
        dec, G, NG = ref.Distance_Decay(M=X, G_array=None)
        pcs, Cor, OE = ref.Get_PCA(distance_bin=dec, M=X, NG_array=NG, SA=True)
        np.testing.assert_array_equal(sf.Cor_Martrix_Dict[name], ref.Refill_Gap(X, np.asarray(Cor), NG, "Cor"))
        np.testing.assert_array_equal(sf.OE_Matrix_Dict[name], ref.Refill_Gap(X, np.asarray(OE), NG, "OE"))
