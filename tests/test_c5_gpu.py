"""C5 at its own size (BASELINE configs[4]: hg19 autosomes at 25 kb, dense
per chromosome) and the compartment eigensolver's edge cases.

chr21 / chr22 (N = 1 926 / 2 053) run the whole compartment path against the
oracle (exact SVD); chr1 (N = 9 971) is checked by sampled correlation columns
against NumPy's corrcoef of the same O/E columns and by eigen-residuals of the
returned components — the oracle's dense SVD of 9 971^2 would take minutes.
Reference: StructureFind.py:201-271 (Distance_Decay), :302-342 (Get_PCA),
:374-423 (Select_PC_new)."""
import warnings

import numpy as np
import pytest

from oracle import structure_ref

pytestmark = pytest.mark.gpu

C5_RES = 25000


def _c5_sizes():
    from hichap_master_amd import synth
    return synth.chrom_bins([synth.HG19[str(c)] for c in range(1, 23)], C5_RES)


def _c5_kw():
    # the bench's C5 generator parameters (bench.c5_synth_kw)
    return dict(A=120.0, trans_density=0.0, comp_block=80, ignore_diags=0, cis_only=True, gap_frac=0.02,
                seed=20201019)


def _c5_matrix(k):
    import torch
    from hichap_master_amd import _lib, ice
    _lib.require_gpu()
    sizes = _c5_sizes()
    buf = torch.empty((sizes[k], sizes[k]), dtype=torch.float64, device="cuda")
    ice.synth_dense(sizes, k, buf.data_ptr(), **_c5_kw())
    torch.cuda.synchronize()
    return buf


def _match_sign(a, b):
    return a * np.sign(np.dot(a, b))


@pytest.mark.parametrize("chrom", [21, 22])
def test_c5_small_autosomes_vs_oracle(chrom):
    from hichap_master_amd.StructureFind import StructureFind
    dM = _c5_matrix(chrom - 1)
    M = dM.cpu().numpy()
    assert M.shape[0] == _c5_sizes()[chrom - 1]
    sf = StructureFind(Res=C5_RES)
    dec, G, NG = sf.Distance_Decay(M=dM, G_array=None)
    d_ref, G_ref, NG_ref = structure_ref.distance_decay(M)
    np.testing.assert_array_equal(NG, NG_ref)
    np.testing.assert_allclose(dec, d_ref, rtol=1e-12)
    pcs, Cor, OE = sf.Get_PCA(distance_bin=dec.copy(), M=dM, NG_array=NG)
    st = sf.pca_status
    assert st["converged"] and st["method"] == "krylov"
    assert st["products"] <= 60, st
    p_ref, C_ref, _ = structure_ref.get_pca(d_ref, M, NG_ref)
    np.testing.assert_allclose(np.asarray(Cor), C_ref, atol=1e-11)
    # PC1 to 1e-11; PC2 / PC3 as far as their eigen-gap allows
    np.testing.assert_allclose(_match_sign(pcs[0], p_ref[0]), p_ref[0], atol=1e-11)
    X = C_ref - C_ref.mean(axis=0)
    s = np.linalg.svd(X, compute_uv=False)
    lam = s ** 2
    for q in (1, 2):
        gap = min(lam[q - 1] - lam[q], lam[q] - lam[q + 1]) / lam[0]
        np.testing.assert_allclose(_match_sign(pcs[q], p_ref[q]), p_ref[q], atol=max(1e-11, 1e-14 / gap))
    np.testing.assert_allclose(st["eigvals"], lam[:3], rtol=1e-12)
    full = sf.compartment(dM)
    ref_full, k_ref, _, _ = structure_ref.compartment(M)
    big = np.abs(ref_full) > 1e-8
    np.testing.assert_array_equal(np.sign(full[big]), np.sign(ref_full[big]))
    np.testing.assert_allclose(full, ref_full, atol=1e-10)


def test_c5_chr1_spot_checks():
    """chr1 at 25 kb (N = 9 971): sampled Cor entries vs NumPy corrcoef of the
    same O/E columns; top-3 components orthonormal with eigen-residuals
    |A v - lambda v| / lambda_1 < 1e-11 (A = Xc^T Xc, Xc = Cor - mean)."""
    from hichap_master_amd.StructureFind import StructureFind
    dM = _c5_matrix(0)
    N = dM.shape[0]
    assert N == 9971
    sf = StructureFind(Res=C5_RES)
    dec, G, NG = sf.Distance_Decay(M=dM, G_array=None)
    pcs, Cor, OE = sf.Get_PCA(distance_bin=dec.copy(), M=dM, NG_array=NG)
    st = sf.pca_status
    assert st["converged"] and st["products"] <= 72, st
    M = dM.cpu().numpy()
    del dM
    C = np.asarray(Cor)
    n = NG.size
    rng = np.random.default_rng(1)
    sel = np.sort(rng.choice(n, size=48, replace=False))
    dd = dec.copy()
    dd[dd == 0] = dd[np.nonzero(dd)].min()
    cols = M[:, NG[sel]]
    dist = np.abs(np.arange(N)[:, None] - NG[sel][None, :])
    oe = np.where(cols != 0, cols / dd[dist], 0.0)
    Cs = structure_ref.pearson_columns(oe)
    np.testing.assert_allclose(C[np.ix_(sel, sel)], Cs, atol=1e-11)
    mu = C.mean(axis=0)
    lam = st["eigvals"]
    for q in range(3):
        v = pcs[q]
        Xv = C @ v - (mu @ v)                          # Xc v = Cor v - 1 (mu . v)
        Av = C.T @ Xv - mu * Xv.sum()                    # Xc^T w = Cor w - mu (1 . w)
        assert np.linalg.norm(Av - lam[q] * v) / lam[0] < 1e-11, q
    np.testing.assert_allclose(pcs @ pcs.T, np.eye(3), atol=1e-12)
    assert lam[0] > lam[1] > lam[2] > 0


def _comp_with_cor(Cor):
    """An hh_comp whose device correlation is ``Cor`` (n x n)."""
    from hichap_master_amd.StructureFind import _Comp
    from hichap_master_amd._lib import call, ptr
    n = Cor.shape[0]
    comp = _Comp(np.eye(n))
    comp.correlation(np.ones(n), np.arange(n))
    call("hh_comp_set_cor", comp.h, ptr(np.ascontiguousarray(Cor)), None)
    return comp


def _planted(n, s, seed):
    """Symmetric matrix with zero column means and eigenvalues s (rest 0.01):
    Xc = Cor, so the PCA components are its top eigenvectors."""
    rng = np.random.default_rng(seed)
    Z = rng.standard_normal((n, n))
    Z -= Z.mean(axis=0)
    U, _ = np.linalg.qr(Z)
    U = U[:, : n - 1]  # orthonormal, orthogonal to 1
    vals = np.full(n - 1, 0.01)
    vals[: len(s)] = s
    return (U * vals) @ U.T, U[:, : len(s)]


def test_pca_planted_spectrum_exact():
    Cor, U = _planted(700, [9.0, 6.0, 4.0, 2.0, 1.5], seed=3)
    comp = _comp_with_cor(Cor)
    pcs, ev, _ = comp.pca(3)
    assert comp.pca_status["converged"]
    for q in range(3):
        np.testing.assert_allclose(_match_sign(pcs[q], U[:, q]), U[:, q], atol=1e-12)
    np.testing.assert_allclose(ev, np.array([9.0, 6.0, 4.0]) ** 2, rtol=1e-12)


def test_pca_near_degenerate_warns():
    """lambda_3 == lambda_4: the third component is not determined, the solver
    must say it did not converge — PC1 / PC2 are still exact."""
    from hichap_master_amd import StructureFind as SFm
    Cor, U = _planted(400, [9.0, 6.0, 4.0, 4.0, 1.0], seed=5)
    comp = _comp_with_cor(Cor)
    old = SFm.PCA_MAX_ITERS
    SFm.PCA_MAX_ITERS = 100
    try:
        with warnings.catch_warnings(record=True) as rec:
            warnings.simplefilter("always")
            pcs, ev, _ = comp.pca(3)
    finally:
        SFm.PCA_MAX_ITERS = old
    assert not comp.pca_status["converged"]
    assert any(issubclass(w.category, RuntimeWarning) for w in rec)
    for q in range(2):
        np.testing.assert_allclose(_match_sign(pcs[q], U[:, q]), U[:, q], atol=1e-11)
    # the third lies in the degenerate plane
    r = pcs[2] - U[:, 2:4] @ (U[:, 2:4].T @ pcs[2])
    assert np.linalg.norm(r) < 1e-10


def test_pca_krylov_matches_subspace_iteration():
    from hichap_master_amd import synth
    from hichap_master_amd._lib import call
    from hichap_master_amd.StructureFind import StructureFind
    rng = np.random.default_rng(44)
    M = synth.dense_chrom(1200, rng, A=90.0, comp_len=(30, 80), gap_frac=0.02).astype(np.float64)
    out = {}
    for meth in (0, 1):
        call("hh_tune", b"pca_method", meth)
        try:
            sf = StructureFind(Res=25000)
            dec, G, NG = sf.Distance_Decay(M=M, G_array=None)
            pcs, Cor, OE = sf.Get_PCA(distance_bin=dec.copy(), M=M, NG_array=NG)
            out[meth] = (pcs, sf.pca_status)
        finally:
            call("hh_tune", b"pca_method", 1)
    assert out[1][1]["method"] == "krylov" and out[0][1]["method"] == "subspace"
    assert out[1][1]["products"] < out[0][1]["products"] / 2
    np.testing.assert_allclose(_match_sign(out[1][0][0], out[0][0][0]), out[0][0][0], atol=1e-11)


def _pca_run(dM, coop):
    from hichap_master_amd._lib import call
    from hichap_master_amd.StructureFind import StructureFind
    call("hh_tune", b"pca_coop", coop)
    try:
        sf = StructureFind(Res=C5_RES)
        dec, G, NG = sf.Distance_Decay(M=dM, G_array=None)
        pcs, Cor, OE = sf.Get_PCA(distance_bin=dec.copy(), M=dM, NG_array=NG)
        return np.asarray(pcs), dict(sf.pca_status)
    finally:
        call("hh_tune", b"pca_coop", 1)


def test_pca_one_launch_orthogonalisation_matches_multilaunch():
    """k_ortho (the Gram-Schmidt + shifted CholeskyQR3 chain of a product in
    one launch, grid barriers between the reductions) against the multi-launch
    chain on C5 chr21: same components / eigenvalues to rounding, and
    bitwise run-to-run (fixed-order reductions)."""
    dM = _c5_matrix(20)
    p0, s0 = _pca_run(dM, 0)
    p1, s1 = _pca_run(dM, 1)
    p2, _ = _pca_run(dM, 1)
    assert s0["converged"] and s1["converged"]
    assert abs(s1["products"] - s0["products"]) <= 8, (s0, s1)
    for q in range(3):
        np.testing.assert_allclose(_match_sign(p1[q], p0[q]), p0[q], atol=1e-11)
    np.testing.assert_allclose(s1["eigvals"], s0["eigvals"], rtol=1e-12)
    np.testing.assert_array_equal(p1, p2)


def test_pca_one_launch_large_rows_per_block():
    """n = 16 500 > 64 blocks x 256 rows: the 512-rows-per-block variant.
    Low-rank planted spectrum with exactly known eigenvectors."""
    n = 16500
    rng = np.random.default_rng(9)
    Z = rng.standard_normal((n, 6))
    Z -= Z.mean(axis=0)
    U, _ = np.linalg.qr(Z)  # orthonormal, orthogonal to 1
    s = np.array([9.0, 6.0, 4.0, 2.0, 1.5, 1.0])
    Cor = (U * (s - 0.01)) @ U.T
    Cor += np.eye(n) * 0.01
    Cor -= 0.01 / n  # 0.01 (I - 1 1^T / n) + U (s - 0.01) U^T: zero column means
    comp = _comp_with_cor(Cor)
    del Cor
    pcs, ev, _ = comp.pca(3)
    assert comp.pca_status["converged"]
    for q in range(3):
        np.testing.assert_allclose(_match_sign(pcs[q], U[:, q]), U[:, q], atol=1e-11)
    np.testing.assert_allclose(ev, s[:3] ** 2, rtol=1e-11)


def _pca_run_sym(dM, sym):
    from hichap_master_amd._lib import call
    from hichap_master_amd.StructureFind import StructureFind
    call("hh_tune", b"cor_sym", sym)
    try:
        sf = StructureFind(Res=C5_RES)
        dec, G, NG = sf.Distance_Decay(M=dM, G_array=None)
        pcs, Cor, OE = sf.Get_PCA(distance_bin=dec.copy(), M=dM, NG_array=NG)
        return np.asarray(pcs), dict(sf.pca_status), NG.size
    finally:
        call("hh_tune", b"cor_sym", 3)


@pytest.mark.parametrize("chrom", [21, 9])
def test_pca_upper_triangle_product_matches_full(chrom):
    """k_cor_sym (Cor V from the upper triangle of 64 x 64 tiles: column
    products of the tiles on and above the diagonal, row products of those
    strictly above) against the full-matrix split-K product: the same
    components / eigenvalues to rounding (corrcoef's Cor is symmetric only up
    to the rounding of its two divisions), and bitwise run-to-run; chr21 and
    chr9 (padded orders 1 920 / 5 504 at this generator's gaps: neither a
    multiple of the 256-row rectangle, so the last range is ragged)."""
    dM = _c5_matrix(chrom - 1)
    p0, s0, n = _pca_run_sym(dM, 0)
    p1, s1, _ = _pca_run_sym(dM, 1)
    p2, _, _ = _pca_run_sym(dM, 1)
    assert s0["converged"] and s1["converged"]
    assert abs(s1["products"] - s0["products"]) <= 8, (s0, s1)
    for q in range(3):
        np.testing.assert_allclose(_match_sign(p1[q], p0[q]), p0[q], atol=1e-11)
    np.testing.assert_allclose(s1["eigvals"], s0["eigvals"], rtol=1e-12)
    np.testing.assert_array_equal(p1, p2)


@pytest.mark.parametrize("chrom", list(range(1, 23)))
def test_c5_selected_pc_vs_oracle(chrom):
    """every C5 autosome (chr1 at N = 9 971 included)
    through the whole compartment call -- Distance_Decay, Get_PCA,
    Select_PC_new -- against the oracle's (np.corrcoef Cor, top-3 by ARPACK
    on the centred matrix, Select_PC_new restated): PC1 to 1e-10 after sign
    alignment, the same selected PC index, and the A/B sign of every bin with
    |PC| > 1e-8 equal (StructureFind.py:302-342, :374-423)."""
    import sys
    from hichap_master_amd.StructureFind import StructureFind
    dM = _c5_matrix(chrom - 1)
    sf = StructureFind(Res=C5_RES)
    dec, G, NG = sf.Distance_Decay(M=dM, G_array=None)
    pcs, Cor, OE = sf.Get_PCA(distance_bin=dec.copy(), M=dM, NG_array=NG)
    assert sf.pca_status["converged"]
    pc = sf.Select_PC_new(Cor, OE[NG], pcs)
    k_gpu = int(np.argmax([abs(np.dot(pc, p)) for p in pcs]))
    full = np.zeros(dM.shape[0])
    full[NG] = pc
    del Cor, OE, sf
    M = dM.cpu().numpy()
    del dM
    ref_full, k_ref, p_ref, _ = structure_ref.compartment(M, solver="eigsh")
    print(f"chr{chrom}: N={M.shape[0]} selected PC{k_ref + 1}", file=sys.stderr, flush=True)
    np.testing.assert_allclose(_match_sign(pcs[0], p_ref[0]), p_ref[0], atol=1e-10)
    assert k_gpu == k_ref
    big = np.abs(ref_full) > 1e-8
    np.testing.assert_array_equal(np.sign(full[big]), np.sign(ref_full[big]))
    np.testing.assert_allclose(full, ref_full, atol=1e-9)


def test_pca_ortho_fallback_and_grid_cap():
    """k_ortho's co-residency: (a) when its grid barrier gives up
    (simulated: hh_tune ortho_abort_test), hh_comp_pca redoes the solve on the
    multi-launch path and reports it -- same components as the multi-launch
    run, bitwise; (b) a lower grid cap (fewer, taller blocks, as on a box with
    more hardware queues) gives the same components to rounding."""
    from hichap_master_amd._lib import call
    dM = _c5_matrix(20)
    p0, s0 = _pca_run(dM, 0)
    # 1: the abort reported after a completed cooperative launch; 2: the
    # abort raised inside the first k_ortho launch (blocks leave their grid
    # barriers early, the workspace is partly written)
    for mode in (1, 2):
        call("hh_tune", b"ortho_abort_test", mode)
        try:
            p1, s1 = _pca_run(dM, 1)
        finally:
            call("hh_tune", b"ortho_abort_test", 0)
        assert s1["ortho_fallback"] and s1["converged"] and not s0["ortho_fallback"]
        np.testing.assert_array_equal(p1, p0)
    call("hh_tune", b"ortho_grid_cap", 8)
    try:
        p2, s2 = _pca_run(dM, 1)
    finally:
        call("hh_tune", b"ortho_grid_cap", 0)
    assert s2["converged"] and not s2["ortho_fallback"]
    for q in range(3):
        np.testing.assert_allclose(_match_sign(p2[q], p0[q]), p0[q], atol=1e-11)


def test_pca_pipelined_upper_triangle_product_bitwise():
    """k_cor_sym_pf (V staged once per rectangle, the next column tile's
    first loads in flight) against k_cor_sym: the same MFMA sequence and
    partial sums, so bitwise the same components (chr9: ragged last range)."""
    dM = _c5_matrix(8)
    p1, s1, _ = _pca_run_sym(dM, 1)
    p2, s2, _ = _pca_run_sym(dM, 2)
    assert s1["products"] == s2["products"]
    np.testing.assert_array_equal(p1, p2)
    # cor_sym 3: the same kernel with whole-line Cor loads (each output
    # column summed over the same rows in the same order): bitwise too
    p3, s3, _ = _pca_run_sym(dM, 3)
    assert s3["products"] == s2["products"]
    np.testing.assert_array_equal(p3, p2)
