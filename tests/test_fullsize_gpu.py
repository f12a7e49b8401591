"""Full-size checks of the structure / correction paths at the configurations
HiCHap runs them (VERDICT r1 "What's weak" 8):

* C2's TAD step: gap + DI scan of hg19 chr1 at 10 kb (N = 24 926, window
  600 kb = 60 bins, minTAD 200 kb) from the ICE-balanced pixel table in HBM,
  against the banded restatement of Get_Gap / Get_DI (StructureFind.py:721-839,
  oracle/structure_ref.get_*_band; N x N would be 5 GB).
* GenomeWideMatrixCorrection at HiCHap's default wholeRes (500 kb) on the
  diploid hg19 layout (2n = 12 174 bins), against oracle/hichap_ref
  (matrixBuilding.py:857-901)."""
import numpy as np
import pytest

from oracle import hichap_ref, structure_ref

pytestmark = pytest.mark.gpu


def test_c2_tad_scan_full_size():
    from hichap_master_amd import _lib, ice
    from hichap_master_amd.StructureFind import StructureFind
    from bench import config
    _lib.require_gpu()
    sizes, kw, label, target, tf = config("c2")
    m = ice.ContactMatrix.synthetic(sizes, **kw)
    w, st = ice.balance_matrix(m, ice.IceOptions())
    assert st["converged"]
    b1, b2, c = m.export_upper()
    m.close()
    N = int(sizes[0])
    assert N == 24926 and b1.size > 4e7
    sf = StructureFind(Res=10000)
    sf.TAD_parameter_init(200000, 4000000, 3, 600000, "ttest")
    gap, di = sf.di_scan_pixels(b1, b2, c, w, 0, N)
    B, lb, win = 60, 20, 60
    band = structure_ref.band_from_pixels(b1, b2, c, w, 0, N, B)
    gref = structure_ref.get_gap_band(band, B, lb)
    np.testing.assert_array_equal(gap, gref)
    dref = structure_ref.get_di_band(band, B, gref, win, "ttest")
    # DI is O(1); near-zero values are differences of nearly equal means, so
    # their absolute rounding (different summation order) is the bound there
    np.testing.assert_allclose(di, dref, rtol=1e-11, atol=1e-13)
    assert np.count_nonzero(di) > 0.9 * (N - gref.size - 2 * win)


def _diploid_inputs(res, seed=17):
    """T (n x n, symmetric) and an asymmetric imputed H (2n x 2n, M then P
    halves) shaped like HaplotypeMatrixBuilding's output."""
    from hichap_master_amd import synth
    rng = np.random.default_rng(seed)
    nb = synth.genome_bins(res)
    b1, b2, c, off = synth.coo_genome(nb, rng, A=400.0, trans_density=0.05)
    n = int(off[-1])
    T = synth.coo_to_dense(b1, b2, c, n).astype(np.int64)
    H = np.zeros((2 * n, 2 * n), dtype=np.int64)
    for (r0, c0, p) in ((0, 0, 0.3), (n, n, 0.3), (0, n, 0.05), (n, 0, 0.05)):
        # independent draws per ordered cell: R1/R2 imputation is asymmetric
        H[r0:r0 + n, c0:c0 + n] = rng.binomial(T, p)
    for k in range(len(nb)):  # a SNP-poor stretch in each M copy
        s = int(off[k])
        H[s:s + 3, :] = rng.binomial(H[s:s + 3, :], 0.02)
    bins = {str(k): (int(off[k]), int(off[k + 1]) - 1) for k in range(len(nb))}
    hap = {}
    for k in range(len(nb)):
        hap["M" + str(k)] = (int(off[k]), int(off[k + 1]) - 1)
        hap["P" + str(k)] = (n + int(off[k]), n + int(off[k + 1]) - 1)
    return bins, hap, T, H


def test_genome_wide_correction_default_wholeres():
    from hichap_master_amd import _lib
    from hichap_master_amd.matrixBuilding import GenomeWideMatrixCorrection
    _lib.require_gpu()
    from hichap_master_amd import synth
    bins, hap, T, H = _diploid_inputs(500000)
    assert H.shape[0] == 2 * sum(synth.genome_bins(500000))
    out = GenomeWideMatrixCorrection(bins, hap, T, H)
    ref = hichap_ref.genome_wide_correction(bins, hap, T, H)
    np.testing.assert_allclose(out, ref, rtol=1e-11, atol=1e-300)
    np.testing.assert_allclose(out.sum(), H.sum(), rtol=1e-9)
