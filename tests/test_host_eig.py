"""The Krylov PCA's Rayleigh-Ritz eigensolver (host C++, hh_sym_topk: Householder
tridiagonalisation + implicit QL + inverse iteration) against numpy.linalg.eigh.
No GPU needed."""
import numpy as np
import pytest

from hichap_master_amd._lib import call, ptr


@pytest.mark.parametrize("m,k", [(16, 16), (40, 16), (64, 16), (96, 16), (128, 3)])
def test_sym_topk_matches_eigh(m, k):
    rng = np.random.default_rng(m)
    X = rng.standard_normal((m + 16, m)) * np.geomspace(1.0, 1e-4, m)
    H = X.T @ X
    ev = np.empty(k)
    Y = np.empty((m, k))
    call("hh_sym_topk", ptr(H), m, k, ptr(ev), ptr(Y))
    w, U = np.linalg.eigh(H)
    w, U = w[::-1][:k], U[:, ::-1][:, :k]
    np.testing.assert_allclose(ev, w, rtol=1e-12, atol=1e-14 * w[0])
    sg = np.sign(np.sum(U * Y, axis=0))
    np.testing.assert_allclose(Y[:, :3] * sg[:3], U[:, :3], atol=1e-12)
    np.testing.assert_allclose(Y.T @ Y, np.eye(k), atol=1e-12)
    # residuals of every returned pair
    assert np.abs(H @ Y - Y * ev).max() < 1e-11 * w[0]


def test_sym_topk_clustered_and_diagonal():
    # exactly diagonal (no reflectors) and a tight cluster
    d = np.array([5.0, 3.0, 3.0 + 1e-9, 1.0, 0.5, 0.25] + [0.1] * 20)
    m = d.size
    ev = np.empty(6)
    Y = np.empty((m, 6))
    call("hh_sym_topk", ptr(np.diag(d)), m, 6, ptr(ev), ptr(Y))
    np.testing.assert_allclose(ev, np.sort(d)[::-1][:6], rtol=1e-13)
    np.testing.assert_allclose(Y.T @ Y, np.eye(6), atol=1e-12)
    assert np.abs(np.diag(d) @ Y - Y * ev).max() < 1e-12


def test_sym_topk_rejects_bad_args():
    from hichap_master_amd._lib import HipLibraryError
    with pytest.raises(HipLibraryError):
        call("hh_sym_topk", ptr(np.eye(4)), 4, 5, ptr(np.empty(5)), ptr(np.empty((4, 5))))
