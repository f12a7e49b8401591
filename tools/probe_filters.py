"""Diagnostic: sweep time with cooler's filters applied (as bench.py) vs none
(as probe_knobs.py) on a bench config.  python tools/probe_filters.py c3"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import config  # noqa: E402
from hichap_master_amd import _lib, ice  # noqa: E402

_lib.load()
_lib.require_gpu()
sizes, kw = config(sys.argv[1] if len(sys.argv) > 1 else "c3")[:2]
m = ice.ContactMatrix.synthetic(sizes, **kw)
for rep in range(2):
    for name, o in (("no filters", ice.IceOptions(tol=0.0, max_iters=1 << 30, mad_max=0, min_nnz=0)),
                    ("filters", ice.IceOptions(tol=0.0, max_iters=1 << 30))):
        st = ice.IceState(m, o)
        if name == "filters":
            st.marg_local(0, None, None); st.filter_nnz(None)
            st.marg_local(1, None, None); st.filter_count_mad(None)
        st.run(3)
        st.run(40)
        ms, n, it = st.last_timing()
        print(f"[{rep}] {name}: sweep {ms / n:.3f} ms iter {it / n:.3f} ms", flush=True)
        st.close()
m.close()
