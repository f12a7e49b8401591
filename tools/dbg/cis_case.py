"""Debug: the 4-chromosome --cis-only case of the construction test where
the GPU balance did not converge on chromosome 2 (bins 101..125)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from hichap_master_amd import _lib, ice
_lib.load(); _lib.require_gpu()
d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "cis_case.npz"))
b1, b2, cnt, off = d["b1"], d["b2"], d["cnt"], d["off"]
n = int(off[-1])
np.set_printoptions(linewidth=200, precision=6)
for mi in (1, 2, 3, 13, 200):
    w, st = ice.balance(b1, b2, cnt, n, off, cis_only=True, max_iters=mi, rescale_marginals=False)
    print(mi, "w[101:125]", w[101:125], "iters", st["iters"], "scale", st["scale"], "var", st.get("var"), flush=True)
# the same chromosome alone, and genome-wide
sel = (b1 >= 101) & (b1 < 125)
w, st = ice.balance(b1[sel] - 101, b2[sel] - 101, cnt[sel], 24, [0, 24], cis_only=True, max_iters=200)
print("alone", w, st["iters"], st["scale"])
