"""Haplotype imputation on the GPU (pair-parser mode 1 through the C-ABI)
against the reference's own imputation (tests/golden/impute_*.npz) and the
oracle.  Integer counts: exact."""
import numpy as np
import pytest

from oracle import impute_ref
from tests.test_impute_oracle import lines, setup

pytestmark = pytest.mark.gpu

CASES = ["impute_1res", "impute_fine"]


@pytest.fixture(scope="module")
def mb():
    from hichap_master_amd import _lib, matrixBuilding
    _lib.require_gpu()
    return matrixBuilding


def _genome_lines(g):
    return bytes(np.asarray(g["genome"], dtype=np.uint8)).decode().splitlines(keepends=True)


@pytest.mark.parametrize("case", CASES)
def test_imputation_matches_reference(mb, golden, case):
    g = golden(case)
    p, genome, UW, UL, IW, IL = setup(g)
    UWlib = {r: {"Bins": None, "Matrix": UW[r]} for r in UW}
    W, L = mb.HaplotypeImputation(bytes(g["text_M_M"]), bytes(g["text_P_P"]), _genome_lines(g), p["wholeRes"],
                                  p["localRes"], p["chroms"], p["region"], p["min"], p["ratio"], UWlib, UL)
    for res in p["wholeRes"]:
        np.testing.assert_array_equal(W[res]["Matrix"], IW[res])
    for res in p["localRes"]:
        for key, M in L[res].items():
            np.testing.assert_array_equal(M, IL[res].get(key, np.zeros_like(M)), err_msg=key)


def test_full_haplotype_builder_matches_reference(mb, golden, tmp_path):
    g = golden("impute_1res")
    p, genome, UW, UL, IW, IL = setup(g)
    files = {}
    for k in ("Bi_Allelic", "M_M", "P_P", "M_P", "P_M"):
        f = tmp_path / f"S_Valid_{k}.bed"
        f.write_bytes(bytes(g["text_" + k]))
        files[k] = str(f)
    ds = mb.HaplotypeMatrixBuilding(files, _genome_lines(g), p["wholeRes"], p["localRes"], p["region"], p["min"],
                                    p["ratio"], p["chroms"])
    for res in p["wholeRes"]:
        np.testing.assert_array_equal(ds["UnImputated_Whole"][res]["Matrix"], UW[res])
        np.testing.assert_array_equal(ds["Imputated_Whole"][res]["Matrix"], IW[res])
    for res in p["localRes"]:
        for key, M in ds["Imputated_Local"][res].items():
            np.testing.assert_array_equal(M, IL[res].get(key, np.zeros_like(M)), err_msg=key)


def test_p_pass_without_stale_window_raises(mb):
    from hichap_master_amd._lib import HipLibraryError
    genome = ["chr1\t5000000\n", "chr2\t5000000\n"]
    UWlib = {500000: {"Bins": None, "Matrix": np.ones((44, 44), dtype=np.int64)}}
    UL = {}
    with pytest.raises(HipLibraryError, match="stale"):
        mb.HaplotypeImputation(b"", b"chr1\t2000000\tchr2\t2500000\tR1\n", genome, [500000], [], ["#"], 1_000_000, 2,
                               0.9, UWlib, UL)
    # the oracle raises the reference's NameError on the same input
    with pytest.raises(NameError):
        impute_ref.impute({"M_M": [], "P_P": ["chr1\t2000000\tchr2\t2500000\tR1\n"]}, {"1": 5000000, "2": 5000000},
                          ["#"], [500000], [], 1_000_000, 2, 0.9, {500000: np.ones((44, 44), dtype=np.int64)}, {})
