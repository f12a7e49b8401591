"""Load balance of the row-sharded C4 sweep: for world sizes 2/4/8, build each
rank's shard on this one GPU in turn (dist.partition_rows, as bench.py does)
and time its sweep (HIP-event registry, 'ice_sweep').  Prints per-rank sweep
ms and max/mean; the slowest rank bounds an N-GPU iteration.
  python tools/probe_shards.py [2,4,8] [1]     (world sizes; second argument 1 = refine)
HH_TUNE="key=value,..." sets hh_tune knobs first.  refine=1: re-partition
once with per-row weights scaled by each shard's measured time per weight
(dist.refine_weights) and measure again."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from hichap_master_amd import _lib, dist, ice  # noqa: E402

_lib.load()
_lib.require_gpu()
for kv in filter(None, os.environ.get("HH_TUNE", "").split(",")):
    k, v = kv.split("=")
    _lib.call("hh_tune", k.encode(), int(v))
sizes, kw, label, target, tf = bench.config("c4")
rc, ru = ice.synth_row_counts(sizes, **kw)


def measure(world, rr, tag):
    ms = []
    for r in range(world):
        m = ice.ContactMatrix.synthetic(sizes, row_range=(int(rr[r]), int(rr[r + 1])), **kw)
        st = ice.IceState(m, ice.IceOptions(tol=0.0, max_iters=1 << 30))
        out = torch.zeros(max(int(rr[r + 1] - rr[r]), 1), dtype=torch.float64, device="cuda")
        st.marg_local(2, out, None)
        _lib.call("hh_ktime_reset")
        _lib.call("hh_ktime_enable", 1)
        for _ in range(5):
            st.marg_local(2, out, None)
        torch.cuda.synchronize()
        _lib.call("hh_ktime_enable", 0)
        t, n = _lib.ktime("ice_sweep")
        per = {}
        for kn in ("k_sweep_ubands", "k_sweep_flat", "k_sweep_tiled", "k_marg"):
            kt, kc = _lib.ktime(kn)
            per[kn] = kt / max(kc, 1) if kc else 0.0
        inf = m.info()
        ms.append(t / max(n, 1))
        print(f"{tag} world={world} rank={r} rows=[{rr[r]},{rr[r+1]}) pixels={ru[rr[r]:rr[r+1]].sum():.4g} "
              f"payload={inf['payload_bytes']/1e9:.2f}GB (flat {inf['payload_bytes_flat']/1e9:.2f}) "
              f"units={inf['n_units']} flat_units={inf['n_units_flat']} sweep={ms[-1]:.3f}ms "
              + " ".join(f"{k[2:]}={v:.3f}" for k, v in per.items()), flush=True)
        st.close()
        m.close()
    print(f"{tag} world={world}: max {max(ms):.3f} ms, mean {np.mean(ms):.3f} ms, "
          f"imbalance {max(ms)/np.mean(ms):.3f}", flush=True)
    return np.array(ms)


worlds = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["2", "4", "8"])]
refine = len(sys.argv) > 2 and sys.argv[2] == "1"
for world in worlds:
    rr = dist.partition_rows(rc, world)
    ms = measure(world, rr, "payload")
    if refine:
        w2 = dist.refine_weights(rc, rr, ms)
        rr2 = dist.partition_rows(w2, world)
        measure(world, rr2, "refined")
