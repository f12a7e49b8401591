"""Host-side glue of the drop-in modules (no GPU needed)."""
import pytest

from oracle import hichap_ref


@pytest.mark.parametrize("names", [["X", "10", "2", "chr1", "Y", "M"], ["3", "1", "2"]])
def test_sort_chromosomes(names):
    from hichap_master_amd.matrixBuilding import Sort_Chromosomes
    assert Sort_Chromosomes(names) == hichap_ref.sort_chromosomes(names)
