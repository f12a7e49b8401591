"""Refill_Gap (StructureFind.py:463-488): the vectorised restatement that
Compartment() uses for Cor_Martrix_Dict / OE_Matrix_Dict against the
reference's loops (oracle), odd and even non-gap counts (the 'OE' branch
transposes inside its loop)."""
import numpy as np
import pytest

from oracle import structure_ref


@pytest.mark.parametrize("N,n", [(9, 6), (10, 7), (12, 12), (40, 31), (1, 1)])
def test_refill_gap_matches_reference_loops(N, n):
    from hichap_master_amd.StructureFind import StructureFind
    rng = np.random.default_rng(N * 100 + n)
    NG = np.sort(rng.choice(N, n, replace=False))
    M = rng.poisson(3.0, (N, N)).astype(float)
    C = rng.standard_normal((n, n))
    C = C + C.T
    OE = rng.standard_normal((N, n))
    sf = StructureFind.__new__(StructureFind)
    np.testing.assert_array_equal(sf.Refill_Gap(M, C, NG, "Cor"), structure_ref.refill_gap(M, C, NG, "Cor"))
    np.testing.assert_array_equal(sf.Refill_Gap(M, OE, NG, "OE"), structure_ref.refill_gap(M, OE, NG, "OE"))
