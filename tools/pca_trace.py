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
    a = ap.parse_args()
    import torch
    from hichap_master_amd import _lib, ice, synth
    from hichap_master_amd.StructureFind import StructureFind
    from bench import c5_synth_kw
    _lib.call("hh_tune", b"pca_debug", 1)
    _lib.call("hh_tune", b"pca_p", a.p)
    sizes = synth.chrom_bins([synth.HG19[str(c)] for c in range(1, 23)], 25000)
    for c in a.chroms:
        buf = torch.empty((sizes[c - 1], sizes[c - 1]), dtype=torch.float64, device="cuda")
        ice.synth_dense(sizes, c - 1, buf.data_ptr(), **c5_synth_kw())
        sf = StructureFind(Res=25000)
        dec, G, NG = sf.Distance_Decay(M=buf, G_array=None)
        sf.Get_PCA(distance_bin=dec, M=buf, NG_array=NG)
        print(f"chr{c}: {sf.pca_status}", flush=True)


if __name__ == "__main__":
    main()
