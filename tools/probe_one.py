"""Minimal C4 sweep driver for PMC passes: build the synthetic C4 matrix, run
a few sweeps at one sweep_nb (argv[1]), print the sweep time."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hichap_master_amd import ice, _lib, synth  # noqa: E402

_lib.load(); _lib.require_gpu()
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 2
sizes = synth.genome_bins(10000, diploid=True)
A, td = synth.calibrate(sizes, 5e9, 0.2)
m = ice.ContactMatrix.synthetic(sizes, A=A, trans_density=td)
st = ice.IceState(m, ice.IceOptions(tol=0.0, max_iters=10**6, mad_max=0, min_nnz=0))
_lib.call("hh_tune", b"sweep_nb", nb)
st.run(1); st.run(3)
ms, n, _ = st.last_timing()
print(f"nb={nb}: sweep {ms / n:.3f} ms", flush=True)
