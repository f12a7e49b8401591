"""Diagnostic: one marginal sweep (b = 1 -> row sums) of the upper-band sweep
against the symmetric band sweep on a C4-density chromosome; prints where
they differ.  python tools/probe_uband.py [n_bins] [band4]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hichap_master_amd import _lib, ice, synth  # noqa: E402

_lib.load()
_lib.require_gpu()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 14637
band4 = int(sys.argv[2]) if len(sys.argv) > 2 else 1
_lib.call("hh_tune", b"band4", band4)
A, td = synth.calibrate(synth.genome_bins(10000, diploid=True), 5e9, 0.2)
kw = dict(A=A, trans_density=td, comp_block=200, seed=20201015)
m = ice.ContactMatrix.synthetic([n], **kw)
inf = m.info()
print("band_w", inf["band_w"], "band_w4", inf["band_w4"], flush=True)
b1, b2, c = m.export_upper()
want = np.bincount(b1, weights=c, minlength=n) + np.bincount(b2, weights=c, minlength=n)
res = {}
for mode in (0, 2):
    _lib.call("hh_tune", b"uband", mode)
    st = ice.IceState(m, ice.IceOptions(tol=0.0, max_iters=10, mad_max=0, min_nnz=0))
    out = torch.zeros(n, dtype=torch.float64, device="cuda")
    st.marg_local(2, out, None)
    torch.cuda.synchronize()
    res[mode] = out.cpu().numpy()
    st.close()
_lib.call("hh_tune", b"uband", 1)
for mode in (0, 2):
    d = res[mode] - want
    bad = np.nonzero(np.abs(d) > 1e-9 * np.abs(want))[0]
    print(f"mode {mode}: {bad.size} rows differ from the exported row sums", flush=True)
    if bad.size:
        print("  first rows", bad[:20].tolist())
        print("  diffs", d[bad[:20]].tolist())
        print("  last rows", bad[-10:].tolist())
        # per-row: which diagonals' counts are missing? try matching the diff to
        # single pixels of the row
        for r in bad[:6]:
            sel = (b1 == r) | (b2 == r)
            dd = np.where(b1[sel] == r, b2[sel] - r, b1[sel] - r)
            cc = c[sel]
            hits = [(int(x), float(y)) for x, y in zip(dd, cc) if abs(y - abs(d[r])) < 1e-9]
            print(f"  row {r}: diff {d[r]:+.1f}, pixels with that count at d =", hits[:12])
