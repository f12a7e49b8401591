"""Per-cycle trace of the Krylov compartment PCA on C5 chromosomes
(measurement helper): python tools/pca_trace.py [chrom ...] [--p P]."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("chroms", nargs="*", type=int, default=[21, 1])
    ap.add_argument("--p", type=int, default=6)
    ap.add_argument("--coop", type=int, default=1)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--debug", type=int, default=1)
    a = ap.parse_args()
    import torch
    from hichap_master_amd import _lib, ice, synth
    from hichap_master_amd.StructureFind import StructureFind
    from bench import c5_synth_kw
    import time
    _lib.call("hh_tune", b"pca_debug", a.debug if a.reps == 1 else 0)
    _lib.call("hh_tune", b"pca_coop", a.coop)
    _lib.call("hh_tune", b"pca_p", a.p)
    sizes = synth.chrom_bins([synth.HG19[str(c)] for c in range(1, 23)], 25000)
    for c in a.chroms:
        buf = torch.empty((sizes[c - 1], sizes[c - 1]), dtype=torch.float64, device="cuda")
        ice.synth_dense(sizes, c - 1, buf.data_ptr(), **c5_synth_kw())
        sf = StructureFind(Res=25000)
        dec, G, NG = sf.Distance_Decay(M=buf, G_array=None)
        for r in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sf.Get_PCA(distance_bin=dec, M=buf, NG_array=NG)
            torch.cuda.synchronize()
            print(f"chr{c} coop={a.coop} rep {r}: Get_PCA {1000 * (time.perf_counter() - t0):.2f} ms", flush=True)
        print(f"chr{c}: {sf.pca_status}", flush=True)


if __name__ == "__main__":
    main()
