"""GPU probe on the C4 synthetic matrix: sweep time per hh_tune setting
(sweep_flags x sweep_nb, plus the streaming / staging ablations)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hichap_master_amd import ice, _lib, synth  # noqa: E402

_lib.load(); _lib.require_gpu()
target = float(sys.argv[1]) if len(sys.argv) > 1 else 5e9
flags = [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else range(8))]
nbs = [int(x) for x in (sys.argv[3].split(",") if len(sys.argv) > 3 else ["4"])]
sizes = synth.genome_bins(10000, diploid=True)
A, td = synth.calibrate(sizes, target, 0.2)


def tune(k, v):
    _lib.call("hh_tune", k.encode(), int(v))


t0 = time.time()
m = ice.ContactMatrix.synthetic(sizes, A=A, trans_density=td)
inf = m.info()
print(f"nnz={inf['nnz_upper']:.4g} payload={inf['payload_bytes']/1e9:.2f} GB u32={inf['n_slots']:.4g} "
      f"u16={inf['n_slots_narrow']:.4g} tiles={inf['n_tiles']} units={inf['n_units']} build={time.time()-t0:.1f}s",
      flush=True)
st = ice.IceState(m, ice.IceOptions(tol=0.0, max_iters=10**6, mad_max=0, min_nnz=0))
for f in flags:
    tune("sweep_flags", f)
    for abl in (0, 1, 2):
        tune("sweep_ablate", abl)
        for nb in (nbs if abl == 0 else nbs[:1]):
            tune("sweep_nb", nb)
            st.run(2); st.run(8)
            ms, n, it_ms = st.last_timing()
            sw = ms / n
            print(f"flags={f} abl={abl} nb={nb}: sweep {sw:.3f} ms  alg {12.0*inf['nnz_upper']/sw/1e6:.0f} GB/s  "
                  f"payload {inf['payload_bytes']/sw/1e6:.0f} GB/s", flush=True)
    tune("sweep_ablate", 0); tune("sweep_nb", 4)
