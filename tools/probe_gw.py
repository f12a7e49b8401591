"""Per-phase device times of the sparse genome-wide correction at the gw
bench's size (HIP-event registry, hh_ktime): python tools/probe_gw.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hichap_master_amd import _lib  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    import torch
    from hichap_master_amd.matrixBuilding import GenomeWideMatrixCorrectionSparse
    import numpy as np
    from hichap_master_amd import ice, synth
    names_c = synth.HG19_ORDER
    nb = synth.genome_bins(10000)
    n = int(np.sum(nb))
    At, tdt = synth.calibrate(nb, 1.5e9, 0.2)  # bench.py --config gw's inputs
    Ah, tdh = synth.calibrate(nb + nb, 1.5e9 / 2.0, 0.2)
    T = ice.SynthPixels(nb, ordered=False, A=At, trans_density=tdt, comp_block=200, ignore_diags=0, seed=20201021)
    H = ice.SynthPixels(nb + nb, ordered=True, A=Ah, trans_density=tdh, comp_block=200, ignore_diags=0,
                        seed=20201022)
    off = np.concatenate([[0], np.cumsum(nb)])
    bins = {c: (int(off[k]), int(off[k + 1]) - 1) for k, c in enumerate(names_c)}
    hap = {}
    for k, c in enumerate(names_c):
        hap["M" + c] = bins[c]
        hap["P" + c] = (n + bins[c][0], n + bins[c][1])
    names = ["gw_check", "gw_stats_to_end", "gw_sort", "gw_marg", "gw_merge0"]

    keep = []

    def step():
        out = GenomeWideMatrixCorrectionSparse(bins, hap, (T.bin1, T.bin2, T.count), (H.bin1, H.bin2, H.count),
                                               device_result=True)
        if os.environ.get("PROBE_KEEP"):  # hold the outputs until the next step has made its own
            keep.append(out)
            del keep[:-1]
        t = time.perf_counter()
        del out
        if os.environ.get("HH_GW_TIMING"):
            print(f"[probe] del out: {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
    step()
    torch.cuda.synchronize()
    stop = []
    if os.environ.get("PROBE_KEEPALIVE"):  # a one-wave spin kernel always queued on a side stream
        import threading
        side = torch.cuda.Stream()

        def spin():
            with torch.cuda.stream(side):
                while not stop:
                    torch.cuda._sleep(2_000_000)
                    side.synchronize()
        th = threading.Thread(target=spin, daemon=True)
        th.start()
    _lib.call("hh_ktime_reset")
    _lib.call("hh_ktime_enable", 1)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    stop.append(1)
    _lib.call("hh_ktime_enable", 0)
    print(f"wall {1e3 * wall:.2f} ms per correction")
    for nm in names:
        ms, n = _lib.ktime(nm)
        print(f"{nm:18s} {ms / max(steps, 1):9.3f} ms per correction ({n} scopes)")


if __name__ == "__main__":
    main()
