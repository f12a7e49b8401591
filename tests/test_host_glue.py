"""Host-side glue of the drop-in modules (no GPU needed)."""
import pytest

from oracle import hichap_ref


@pytest.mark.parametrize("names", [["X", "10", "2", "chr1", "Y", "M"], ["3", "1", "2"]])
def test_sort_chromosomes(names):
    from hichap_master_amd.matrixBuilding import Sort_Chromosomes
    assert Sort_Chromosomes(names) == hichap_ref.sort_chromosomes(names)


@pytest.mark.parametrize("N,B", [(1, 0), (5, 2), (5, 7), (40, 9)])
def test_column_band_layout(N, B):
    """band[B + k, j] = M[j + k, j] (0 outside): what hh_gap_scan / hh_di_scan read."""
    import numpy as np
    from hichap_master_amd.StructureFind import column_band
    M = np.random.default_rng(N).random((N, N))
    band = column_band(M, B)
    assert band.shape == (2 * B + 1, N)
    for j in range(N):
        for k in range(-B, B + 1):
            want = M[j + k, j] if 0 <= j + k < N else 0.0
            assert band[B + k, j] == want
