"""Host pieces of the file-driven drivers (CPU): the CallPeaks band built
from cooler's pixel table equals the band of the dense fetch
(StructureFind.py:2006-2032), for traditional and allelic data, and the lazy
Matrix_Dict view of the pixel Data_preprocess behaves like a dict."""
import numpy as np
import pytest

from hichap_master_amd import coolio, loops


def _dense_case(seed, N):
    rng = np.random.default_rng(seed)
    H = np.triu(rng.poisson(3.0 * (np.arange(N)[None, :] - np.arange(N)[:, None] + 1.0).clip(1) ** -0.9,
                            size=(N, N)))
    H[7, :] = H[:, 7] = 0
    r, c = np.nonzero(H)
    w = rng.uniform(0.5, 2.0, N)
    w[7] = np.nan
    return H + np.triu(H, 1).T, (r, c, H[r, c]), w


@pytest.mark.parametrize("allelic", [False, True])
@pytest.mark.parametrize("res,N", [(20000, 300), (10000, 260)])
def test_pixel_band_equals_dense_band(allelic, res, N):
    H, (r, c, v), w = _dense_case(res + N, N)
    lo = 1000  # global ids: the chromosome starts at bin 1000
    raw = loops.raw_band_from_pixels(r + lo, c + lo, v, lo, N, loops.band_width(res))
    A = loops.bands(H, None if allelic else w, res, allelic)
    B = loops.bands(None, None if allelic else w, res, allelic, raw=raw)
    assert A.keys() == B.keys()
    for k in A:
        if isinstance(A[k], np.ndarray):
            np.testing.assert_array_equal(A[k], B[k])
        else:
            assert A[k] == B[k]


def test_lazy_matrices(tmp_path):
    from hichap_master_amd.tads import _LazyMatrices
    rng = np.random.default_rng(1)
    cs = [("a", 30 * 10000), ("b", 20 * 10000)]
    i, j = np.triu_indices(50)
    keep = rng.random(i.size) < 0.3
    p = str(tmp_path / "x.cool")
    coolio.create_cooler(p, {10000: (cs, i[keep], j[keep], rng.integers(1, 9, keep.sum()).astype(np.int32))})
    L = _LazyMatrices(f"{p}::10000", ["a", "b"], False)
    assert list(L) == ["a", "b"] and len(L) == 2 and "a" in L and "c" not in L
    with coolio.Cooler(f"{p}::10000") as c:
        np.testing.assert_array_equal(L["b"], c.matrix(balance=False).fetch("b"))
    with pytest.raises(KeyError):
        L["c"]
