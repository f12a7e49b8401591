"""Debug: one sweep at b = 1 with the column-grouped flat kernel, upper tiles
on/off, against the exported table's row sums."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from hichap_master_amd import _lib, ice, synth
_lib.load(); _lib.require_gpu()
rng = np.random.default_rng(41)
b1, b2, c, off = synth.coo_genome([9000, 7000, 600], rng, A=3.0, trans_density=0.0005)
n = int(off[-1])
for fm, fc, up, waves in [(24, 1, 0, 8), (24, 1, 1, 8), (24, 1, 1, 11), (24, -1, 1, 8), (255, 1, 1, 8)]:
    _lib.call("hh_tune", b"flat_max", fm)
    _lib.call("hh_tune", b"flat_cols", fc)
    _lib.call("hh_tune", b"upper_tiles", up)
    _lib.call("hh_tune", b"flatw_waves_up", waves)
    m = ice.ContactMatrix.from_pixels(b1, b2, c, n, off)
    inf = m.info()
    e1, e2, ec = m.export_upper()
    want = np.bincount(e1, weights=ec, minlength=n) + np.bincount(e2, weights=ec, minlength=n)
    st = ice.IceState(m, ice.IceOptions(tol=0.0, max_iters=10, mad_max=0, min_nnz=0))
    out = torch.zeros(n, dtype=torch.float64, device="cuda")
    st.marg_local(2, out, None)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    bad = np.flatnonzero(got != want)
    print(f"flat_max={fm} flat_cols={fc} upper={up} waves={waves} info upper={inf['upper']} units_flat={inf['n_units_flat']} "
          f"bad={bad.size}", flush=True)
    if bad.size:
        d = got[bad] - want[bad]
        print("  first bad", bad[:20].tolist(), "diff", d[:20].tolist())
        print("  by 512-block", np.unique(bad // 512, return_counts=True))
        print("  by 4096-tile", np.unique(bad // 4096, return_counts=True), "sum diff", d.sum())
        # what the column side of strictly upper entries would give per column
        Jr, Jc = e1 >> 12, e2 >> 12
        su = np.bincount(e2[Jc > Jr], weights=ec[Jc > Jr], minlength=n)
        print("  upper col side at bad", su[bad[:20]].tolist())
    st.close(); m.close()
