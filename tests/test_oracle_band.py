"""The banded restatement of Get_Gap / Get_DI (oracle, used for full-size
checks where N x N does not fit) equals the dense restatement, which the
reference's golden vectors pin (test_oracle_golden.py)."""
import numpy as np
import pytest

from hichap_master_amd import synth
from oracle import structure_ref as sr


@pytest.mark.parametrize("test_type", ["ttest", "chitest"])
def test_band_scan_equals_dense(test_type):
    rng = np.random.default_rng(4)
    b1, b2, c, off = synth.coo_genome([400, 300], rng, A=25.0, trans_density=0.01)
    w = np.exp(rng.normal(0, 0.2, size=int(off[-1])))
    w[rng.random(w.size) < 0.03] = np.nan
    lo, N = int(off[1]), int(off[2] - off[1])
    B, lb, win = 12, 5, 10
    band = sr.band_from_pixels(b1, b2, c, w, lo, N, B)
    sel = (b1 >= lo) & (b2 >= lo)
    M = np.zeros((N, N))
    v = c[sel] * w[b1[sel]] * w[b2[sel]]
    M[b1[sel] - lo, b2[sel] - lo] = v
    M[b2[sel] - lo, b1[sel] - lo] = v
    M = np.nan_to_num(M)
    gd = sr.get_gap(M, lb * 10000, 10000)
    np.testing.assert_array_equal(sr.get_gap_band(band, B, lb), gd)
    np.testing.assert_array_equal(sr.get_di_band(band, B, gd, win, test_type), sr.get_di(M, gd, win, test_type))
