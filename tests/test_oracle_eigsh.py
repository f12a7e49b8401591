"""The oracle's large-n PCA (ARPACK on A = Xc^T Xc, matrix-vector products
only) equals its exact-SVD form (golden-pinned) on the same correlation:
components to 1e-12, the same selected PC.  This is what pins chr1 at C5's
size without a dense SVD of 9 971^2."""
import numpy as np

from hichap_master_amd import synth
from oracle import structure_ref as sr


def test_eigsh_components_equal_exact_svd(golden):
    for M in (golden("compartment_n150")["M"],
              synth.dense_chrom(900, np.random.default_rng(3), A=90.0, comp_len=(30, 80),
                                gap_frac=0.02).astype(float)):
        a = sr.compartment(M)
        b = sr.compartment(M, solver="eigsh")
        assert a[1] == b[1]
        np.testing.assert_allclose(b[2], a[2], atol=1e-12)
        np.testing.assert_allclose(b[0], a[0], atol=1e-12)
