"""GPU probe: synthetic matrix generation + ICE sweep timing per variant."""
import sys, time
import numpy as np
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hichap_master_amd import ice, _lib, synth

_lib.load(); _lib.require_gpu()
name = sys.argv[1]
target = float(sys.argv[2])
if name == "c2":
    sizes = [24926]; A, td = synth.calibrate(sizes, target)
elif name == "c4":
    sizes = synth.genome_bins(10000, diploid=True); A, td = synth.calibrate(sizes, target, 0.2)
elif name == "wgcis":
    sizes = synth.genome_bins(10000, diploid=True); A, td = synth.calibrate(sizes, target, 0.0)
kw = dict(A=A, trans_density=td)
t0 = time.time()
rc, ru = ice.synth_row_counts(sizes, **kw)
t1 = time.time()
m = ice.ContactMatrix.synthetic(sizes, **kw)
t2 = time.time()
inf = m.info()
print(f"{name}: A={A:.1f} td={td:.3g} n={inf['n_bins']} nnz_upper={inf['nnz_upper']:.4g} entries={inf['n_entries']:.4g} "
      f"slots={inf['n_slots']:.4g} fill={inf['n_entries']/max(inf['n_slots'],1):.3f} tiles={inf['n_tiles']} units={inf['n_units']} "
      f"bytes={inf['device_bytes']/1e9:.2f}GB count={t1-t0:.2f}s build={t2-t1:.2f}s", flush=True)
st = ice.IceState(m, ice.IceOptions(tol=0.0, max_iters=10**6, mad_max=0, min_nnz=0))
def run(label):
    st.run(2)
    st.run(10)
    ms, n, it_ms = st.last_timing()
    sw = ms / n
    alg = 12.0 * inf["nnz_upper"]
    real = float(inf["payload_bytes"])
    print(f"  {label:28s} sweep {sw:.3f} ms  iter {it_ms/n:.3f} ms  it/s {1000*n/it_ms:.1f}  "
          f"alg {alg/sw/1e6:.0f} GB/s  real {real/sw/1e6:.0f} GB/s", flush=True)

run("tiled")
run("tiled")
