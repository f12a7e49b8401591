"""GPU probe on C4-sized synthetic matrices: sweep time per knob setting."""
import sys, time
import numpy as np
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hichap_master_amd import ice, _lib, synth

_lib.load(); _lib.require_gpu()
target = float(sys.argv[1]) if len(sys.argv) > 1 else 5e9
units = [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["131072"])]
sizes = synth.genome_bins(10000, diploid=True)
A, td = synth.calibrate(sizes, target, 0.2)
kw = dict(A=A, trans_density=td)

def tune(k, v):
    _lib.call("hh_tune", k.encode(), int(v))

for ue in units:
    tune("unit_entries", ue)
    t0 = time.time()
    m = ice.ContactMatrix.synthetic(sizes, **kw)
    inf = m.info()
    print(f"unit_entries={ue}: nnz={inf['nnz_upper']:.4g} slots={inf['n_slots']:.4g} tiles={inf['n_tiles']} "
          f"units={inf['n_units']} build={time.time()-t0:.1f}s", flush=True)
    st = ice.IceState(m, ice.IceOptions(tol=0.0, max_iters=10**6, mad_max=0, min_nnz=0))
    for abl in (0, 1, 2):
        tune("sweep_ablate", abl)
        for nb in ((1, 2, 4, 8) if abl == 0 else (4,)):
            tune("sweep_nb", nb)
            st.run(2); st.run(8)
            ms, n, it_ms = st.last_timing()
            sw = ms / n
            print(f"  abl={abl} nb={nb}: sweep {sw:.3f} ms  it/s {1000*n/it_ms:.1f}  "
                  f"alg {12.0*inf['nnz_upper']/sw/1e6:.0f} GB/s  real {inf['payload_bytes']/sw/1e6:.0f} GB/s", flush=True)
    tune("sweep_ablate", 0); tune("sweep_nb", 4)
    st.close(); m.close()
