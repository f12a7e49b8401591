"""GPU probe on the C4 synthetic matrix: ICE sweep time under run-time knob
settings (hh_tune), one matrix build.  Usage:
    python tools/probe_knobs.py "band_concurrent=0" "band_concurrent=1,sweep_nb=1" ...
Build-time knobs (band_w, unit_entries) may be given with --build k=v,..."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hichap_master_amd import ice, _lib, synth  # noqa: E402


def tune(spec):
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=")
        _lib.call("hh_tune", k.encode(), int(v))


ap = argparse.ArgumentParser()
ap.add_argument("settings", nargs="+")
ap.add_argument("--build", default="")
ap.add_argument("--nnz", type=float, default=5e9)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--config", default="", help="a bench.py config (c2, c3, ...) instead of C4")
ap.add_argument("--shard", default="", help="k/N: build only shard k of N (equal 512-row blocks)")
ap.add_argument("--stream", action="store_true", help="first the read rates of the matrix's own buffers "
                "(hh_matrix_stream_probe: linear reads; the flat tiles streamed in the flat sweep's order)")
a = ap.parse_args()
_lib.load(); _lib.require_gpu()
if a.config:
    from bench import config
    sizes, kw = config(a.config)[:2]
else:
    sizes = synth.genome_bins(10000, diploid=True)
    A, td = synth.calibrate(sizes, a.nnz, 0.2)
    kw = dict(A=A, trans_density=td)
tune(a.build)
t0 = time.time()
if a.shard:
    k, N = map(int, a.shard.split("/"))
    nrb = (int(sum(sizes)) + 511) // 512
    kw["row_range"] = (min(int(sum(sizes)), k * nrb // N * 512), min(int(sum(sizes)), (k + 1) * nrb // N * 512))
m = ice.ContactMatrix.synthetic(sizes, **kw)
inf = m.info()
print(f"build {time.time()-t0:.1f}s band_w={inf['band_w']} band_w4={inf['band_w4']} units={inf['n_units']} "
      f"payload {inf['payload_bytes']/1e9:.2f} GB (flat {inf['payload_bytes_flat']/1e9:.2f} GB in "
      f"{inf['n_units_flat']} units, band {(2 * inf['band_w'] + 16) * (inf['row_hi'] - inf['row_lo']) / 1e9:.2f} GB, band4 "
      f"{(inf['band_w4'] - inf['band_w'] + 32) * (inf['band_w4'] > inf['band_w']) * (inf['row_hi'] - inf['row_lo']) / 1e9:.2f} GB) "
      f"tiles {inf['n_tiles']}", flush=True)
if a.stream:
    import ctypes as C
    out = (C.c_double * 20)()
    names = ["wide tile entries", "narrow tile entries", "uint8 band", "nibble band",
             "flat tiles, 11 waves, 1 block/CU", "flat tiles, 11 waves", "flat tiles, 16 waves",
             "flat tiles coalesced, 11 waves, 1 block/CU", "flat tiles coalesced, 8 waves",
             "narrow tile entries, lane-major runs"]
    for rep in range(2):
        _lib.call("hh_matrix_stream_probe", m.handle, 5, out, 20)
        for i, nm in enumerate(names):
            if out[2 * i + 1] > 0:
                print(f"[stream {rep}] {nm}: {out[2*i+1]/1e9:.3f} GB in {out[2*i]:.3f} ms = "
                      f"{out[2*i+1]/out[2*i]/1e9:.2f} TB/s", flush=True)
st = ice.IceState(m, ice.IceOptions(tol=0.0, max_iters=10**6, mad_max=0, min_nnz=0))
def run_shard(n):
    """A shard cannot use hh_ice_run: one-rank sharded loop, wall time."""
    import ctypes as C
    import numpy as np
    rr = np.array([0, int(sum(sizes))], np.int64)
    _lib.call("hh_ice_run_sharded", st._h, 1, _lib.ptr(rr), None, None, int(n), None)


for rep in range(2):
    for spec in a.settings:
        if "uband=" in spec:  # create-time knob: a new ICE state
            st.close()
            tune(spec)
            st = ice.IceState(m, ice.IceOptions(tol=0.0, max_iters=10**6, mad_max=0, min_nnz=0))
        tune(spec)
        if a.shard:
            run_shard(2)
            t0 = time.perf_counter()
            run_shard(a.iters)
            print(f"[{rep}] {spec}: shard iter {(time.perf_counter() - t0) * 1e3 / a.iters:.3f} ms (wall)", flush=True)
            continue
        st.run(2)
        st.run(a.iters)
        ms, n, it_ms = st.last_timing()
        print(f"[{rep}] {spec}: sweep {ms/n:.3f} ms  iter {it_ms/n:.3f} ms", flush=True)
st.close(); m.close()
