import sys, time
sys.path.insert(0, '.')
import numpy as np
from hichap_master_amd import ice, synth
for res, target, dip in [(40000, 8e8, False), (10000, 5e9, True)]:
    sizes = synth.genome_bins(res, diploid=dip)
    A, td = synth.calibrate(sizes, target, 0.2)
    kw = dict(A=A, trans_density=td, comp_block=200, seed=20201015)
    m = ice.ContactMatrix.synthetic(sizes, **kw)
    for it in (200, 1000, 3000):
        t = time.time()
        w, st = ice.balance_matrix(m, ice.IceOptions(max_iters=it))
        print(res, it, {k: st[k] for k in ('var', 'iters', 'converged', 'scale')}, np.isnan(w).sum(), round(time.time() - t, 2), flush=True)
    m.close()
