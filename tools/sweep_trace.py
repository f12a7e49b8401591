"""Block timeline of the single-launch ICE sweep (k_sweep_all) on a bench
config: per body (tiled units / band blocks / flat units) the block count,
block duration percentiles and the span; the CUs' busy fraction; and the
launch's critical tail (blocks still running in its last 20 %).  Diagnostic
only (hh_tune "sweep_trace").  Usage:
    python tools/sweep_trace.py --config c2 [--build unit_entries=..] [knob=v,...]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hichap_master_amd import ice, _lib  # noqa: E402


def tune(spec):
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=")
        _lib.call("hh_tune", k.encode(), int(v))


ap = argparse.ArgumentParser()
ap.add_argument("settings", nargs="*", default=[""])
ap.add_argument("--config", default="c2")
ap.add_argument("--build", default="")
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
_lib.load(); _lib.require_gpu()
from bench import config  # noqa: E402
sizes, kw = config(a.config)[:2]
tune(a.build)
m = ice.ContactMatrix.synthetic(sizes, **kw)
inf = m.info()
n_units, n_flat = inf["n_units"], inf["n_units_flat"]
print(f"units {n_units} (flat {n_flat}) tiles {inf['n_tiles']} payload {inf['payload_bytes']/1e6:.1f} MB", flush=True)
_lib.call("hh_tune", b"sweep_trace", 1 << 20)
for spec in a.settings or [""]:
    tune("sweep_single=1," + spec)
    st = ice.IceState(m, ice.IceOptions(tol=0.0, max_iters=10**6, mad_max=0, min_nnz=0))
    import ctypes as C
    spans, rows = [], []
    for it in range(a.iters):
        _lib.call("hh_ice_run", st._h, 1, None)
        n = C.c_int64()
        _lib.call("hh_sweep_trace", None, 0, C.byref(n))
        buf = np.zeros(3 * n.value, np.uint64)
        _lib.call("hh_sweep_trace", _lib.ptr(buf), buf.size, C.byref(n))
        tr = buf.reshape(-1, 3).astype(np.int64)
        if it >= 3:
            rows.append(tr)
    n_tiled = n_units - n_flat
    n_band = rows[0].shape[0] - n_units
    print(f"[{spec or 'default'}] grid {rows[0].shape[0]} = tiled {n_tiled} | band {n_band} | flat {n_flat}")
    sp = []
    for tr in rows:
        t0 = tr[:, 0].min()
        sp.append((tr[:, 1].max() - t0) / 100.0)  # 100 MHz ticks -> us
    print(f"  span us: median {np.median(sp):.1f} min {np.min(sp):.1f}")
    tr = rows[int(np.argsort(sp)[len(sp) // 2])]
    t0 = tr[:, 0].min()
    s, e = (tr[:, 0] - t0) / 100.0, (tr[:, 1] - t0) / 100.0
    d = e - s
    span = e.max()
    kinds = {"tiled": slice(0, n_tiled), "band": slice(n_tiled, n_tiled + n_band),
             "flat": slice(n_tiled + n_band, tr.shape[0])}
    for k, sl in kinds.items():
        if sl.stop <= sl.start:
            continue
        dd = d[sl]
        print(f"  {k:5s} n={dd.size:5d} dur us p50 {np.percentile(dd,50):6.2f} p90 {np.percentile(dd,90):6.2f} "
              f"max {dd.max():6.2f} sum {dd.sum():9.1f}  start p50 {np.percentile(s[sl],50):6.1f} "
              f"last end {e[sl].max():6.1f}")
    cu = tr[:, 2]
    busy = np.zeros(int(cu.max()) + 1)
    np.add.at(busy, cu, d)
    print(f"  CUs seen {np.count_nonzero(busy)}; block-us per CU: mean {busy[busy>0].mean():.1f} "
          f"max {busy.max():.1f}; block-us total / (span x CUs x 2 slots) = {d.sum() / (span * np.count_nonzero(busy) * 2):.2f}")
    late = e > 0.8 * span
    for k, sl in kinds.items():
        idx = np.arange(tr.shape[0])[sl]
        nl = np.count_nonzero(late[idx])
        if nl:
            print(f"  {k}: {nl} blocks end in the last 20 % (latest starts {s[idx][late[idx]].max():.1f} us, "
                  f"longest {d[idx][late[idx]].max():.1f} us)")
    # concurrency profile in 10 bins
    edges = np.linspace(0, span, 11)
    conc = [np.count_nonzero((s < edges[i + 1]) & (e > edges[i])) for i in range(10)]
    print("  blocks live per tenth of the span:", conc)
    st.close() if hasattr(st, "close") else None
