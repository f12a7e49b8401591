"""GPU probe on the C4 synthetic matrix: sweep time (tiles + band) per
build-time plan (unit_entries, band_w) and sweep_nb."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hichap_master_amd import ice, _lib, synth  # noqa: E402

_lib.load(); _lib.require_gpu()
sizes = synth.genome_bins(10000, diploid=True)
A, td = synth.calibrate(sizes, 5e9, 0.2)


def tune(k, v):
    _lib.call("hh_tune", k.encode(), int(v))


for band_w in [int(x) for x in sys.argv[1].split(",")]:
    for ue in [int(x) for x in sys.argv[2].split(",")]:
        tune("band_w", band_w)
        tune("unit_entries", ue)
        t0 = time.time()
        m = ice.ContactMatrix.synthetic(sizes, A=A, trans_density=td)
        inf = m.info()
        st = ice.IceState(m, ice.IceOptions(tol=0.0, max_iters=10**6, mad_max=0, min_nnz=0))
        for nb in [int(x) for x in sys.argv[3].split(",")]:
            tune("sweep_nb", nb)
            st.run(2); st.run(8)
            ms, n, it_ms = st.last_timing()
            print(f"band_w={inf['band_w']} unit_entries={ue} units={inf['n_units']} nb={nb}: sweep {ms/n:.3f} ms "
                  f"payload {inf['payload_bytes']/1e9:.2f} GB build {time.time()-t0:.1f}s", flush=True)
        st.close(); m.close()
tune("band_w", -1); tune("unit_entries", 0); tune("sweep_nb", 2)
