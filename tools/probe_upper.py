"""Timing probe of the C4 sweep per kernel (HIP-event registry, one stream and
the default three streams) for build-time layout knobs, e.g. the
upper-triangle tiles (hh_tune upper_tiles) with the library of the current
column-tile width (HH_LIB selects another build, e.g. -DHH_KWBITS=12).
    python tools/probe_upper.py "upper_tiles=0" "upper_tiles=1"
Timing only: with upper_tiles=1 and no column side the marginals are wrong."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hichap_master_amd import _lib, ice, synth  # noqa: E402

_lib.load()
_lib.require_gpu()
sizes = synth.genome_bins(10000, diploid=True)
A, td = synth.calibrate(sizes, 5e9, 0.2)
kw = dict(A=A, trans_density=td, comp_block=200, seed=20201015)


def tune(spec):
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=")
        _lib.call("hh_tune", k.encode(), int(v))


for spec in sys.argv[1:]:
    tune(spec)
    t0 = time.time()
    m = ice.ContactMatrix.synthetic(sizes, **kw)
    inf = m.info()
    print(f"{spec} lib={os.path.basename(_lib.LIB_PATH)} build {time.time() - t0:.1f}s payload "
          f"{inf['payload_bytes'] / 1e9:.2f} GB (flat {inf['payload_bytes_flat'] / 1e9:.2f}) tiles {inf['n_tiles']} "
          f"units {inf['n_units']} flat_units {inf['n_units_flat']}", flush=True)
    st = ice.IceState(m, ice.IceOptions(tol=0.0, max_iters=1 << 30, mad_max=0, min_nnz=0))
    out = torch.zeros(int(sum(sizes)), dtype=torch.float64, device="cuda")
    for conc in (0, 1):
        _lib.call("hh_tune", b"band_concurrent", conc)
        st.marg_local(2, out)
        _lib.call("hh_ktime_reset")
        _lib.call("hh_ktime_enable", 1)
        for _ in range(10):
            st.marg_local(2, out)
        torch.cuda.synchronize()
        _lib.call("hh_ktime_enable", 0)
        per = {}
        for kn in ("ice_sweep", "k_sweep_ubands", "k_sweep_flat", "k_sweep_tiled", "k_marg"):
            t, n = _lib.ktime(kn)
            per[kn] = t / n if n else 0.0
        print(f"  conc={conc} " + " ".join(f"{k}={v:.3f}" for k, v in per.items()), flush=True)
    _lib.call("hh_tune", b"band_concurrent", 1)
    st.close()
    m.close()
