"""Degenerate synthetic check: hg19 chr21+chr22 at 40 kb with C3's saturated
calibration (A = 1e6) -- oracle vs GPU ICE trajectories."""
import sys
sys.path.insert(0, '.')
import numpy as np
from hichap_master_amd import ice, synth
from oracle import ice_ref
sizes = synth.genome_bins(40000, chroms=["21", "22"])
for A, td in [(1e6, 0.0557), (3e3, 0.0557)]:
    rng = np.random.default_rng(3)
    b1, b2, c, off = synth.coo_genome(list(sizes), rng, A=A, trans_density=td)
    n = int(off[-1])
    for it in (50, 200, 1000):
        w, st = ice.balance(b1, b2, c, n, off, max_iters=it)
        wr, sr = ice_ref.balance(b1, b2, c, n, off, max_iters=it)
        ok = ~np.isnan(wr)
        print(A, it, "gpu", st["var"], st["iters"], "oracle", sr["var"], sr["iters"],
              "maxrel", float(np.max(np.abs(w[ok] - wr[ok]) / np.abs(wr[ok]))), "cmax", c.max(), flush=True)
