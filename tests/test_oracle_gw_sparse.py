"""oracle/hichap_ref.genome_wide_correction_sparse (the pixel-table restatement
of GenomeWideMatrixCorrection, matrixBuilding.py:857-901) against the
reference's own dense output (golden genomewide_3chrom) and the dense oracle
on random asymmetric H with orphan cells, diagonals, empty rows and gaps."""
import numpy as np
import pytest

from oracle import hichap_ref


def _tables(T, H):
    i, j = np.nonzero(np.triu(T))
    r, c = np.nonzero(H)
    return (i, j, T[i, j]), (r, c, H[r, c])


def _layout(names, sizes):
    n = sum(sizes)
    bins, hbins, s = {}, {}, 0
    for nm, L in zip(names, sizes):
        bins[nm] = (s, s + L - 1)
        hbins["M" + nm] = (s, s + L - 1)
        hbins["P" + nm] = (n + s, n + s + L - 1)
        s += L
    return bins, hbins


def _check(b1, b2, v, dense, rtol):
    N = dense.shape[0]
    key = b1 * N + b2
    assert np.all(b1 <= b2) and np.all(np.diff(key) > 0)
    np.testing.assert_allclose(v, dense[b1, b2], rtol=rtol, atol=0)
    iu, ju = np.nonzero(np.triu(dense))
    assert np.array_equal(np.sort(iu * N + ju), np.sort(key[v != 0]))


def test_sparse_oracle_matches_reference_golden(golden):
    g = golden("genomewide_3chrom")
    bins, hbins = _layout([str(x) for x in g["names"]], [int(x) for x in g["sizes"]])
    tp, hc = _tables(g["T_M"], g["H_M"])
    _check(*hichap_ref.genome_wide_correction_sparse(bins, hbins, tp, hc), g["Nor"], 1e-12)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_sparse_oracle_matches_dense_oracle(seed):
    rng = np.random.default_rng(seed)
    sizes = [70, 45, 90, 30]
    n = sum(sizes)
    T = np.triu(rng.poisson(2.0, size=(n, n)) * (rng.random((n, n)) < 0.5))
    T = T + np.triu(T, 1).T
    T[5, :] = T[:, 5] = 0
    H = rng.poisson(0.8, size=(2 * n, 2 * n)) * (rng.random((2 * n, 2 * n)) < 0.3)
    H[10, :] = 0
    H[:, 33] = 0
    bins, hbins = _layout(["1", "2", "10", "X"], sizes)
    tp, hc = _tables(T, H)
    dense = hichap_ref.genome_wide_correction(bins, hbins, T, H)
    _check(*hichap_ref.genome_wide_correction_sparse(bins, hbins, tp, hc), dense, 1e-12)
