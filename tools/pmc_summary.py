"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs into a per-kernel
JSON (profiles/*_pmc.json) that bench.py reads for roofline.traffic.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts
128-B requests of wide coalesced streaming reads as 64 B, i.e. reports half
the bytes; WRITE_SIZE is exact for 16-B/lane stores.  traffic_bytes =
2 * FETCH_SIZE + WRITE_SIZE (both in KiB units in the CSV).

  pmc_summary.py fetch.csv write.csv out.json [commit] [real_bytes_per_sweep] [line bench.log]

With `line` (c4 | c4h | c3 | c2 | cis | gw | c5 | twostep | twostep_genome) and the profiled bench's log, _meta records the
sources' fingerprint (bench.src_sha) and the workload of that run, so bench.py
reports the traffic only for runs of the same build on the same workload."""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOAD_KEYS = {"c4": ("n_bins", "nnz_upper"), "gw": ("T_pixels", "H_cells"),
                 "c5": ("workload", "n_chroms", "bins_total"),
                 "twostep": ("workload", "N"), "twostep_genome": ("workload", "bins", "sum_N2"),
                 **{k: ("n_bins", "nnz_upper") for k in ("c4h", "c3", "c2", "cis")}}


def load(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main(fetch_csv, write_csv, out, commit=None, real_bytes_per_sweep=None, line=None, bench_log=None):
    """Optional metadata: the commit the profiled build came from, the
    layout's payload bytes per sweep (bench.py scales traffic to shards by it),
    and (line, bench_log) the source fingerprint + workload of the run."""
    (f, nf), (w, _) = load(fetch_csv, "FETCH_SIZE"), load(write_csv, "WRITE_SIZE")
    res = {}
    meta = {"commit": commit,
            "real_bytes_per_sweep": float(real_bytes_per_sweep) if real_bytes_per_sweep not in (None, "", "-") else None}
    if line:
        sys.path.insert(0, ROOT)
        import bench
        meta["line"] = line
        meta["src_sha"] = bench.src_sha(line)
        cfg = json.loads(open(bench_log).read().strip().splitlines()[-1])["config"]
        meta["workload"] = {k: cfg[k] for k in WORKLOAD_KEYS[line]}
    res["_meta"] = meta
    for k in sorted(set(f) | set(w)):
        fb, wb = f.get(k, 0.0) * 1024.0, w.get(k, 0.0) * 1024.0
        res[k] = {"fetch_size_bytes": fb, "write_size_bytes": wb, "traffic_bytes": 2.0 * fb + wb,
                  "dispatches": nf.get(k, 0)}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        if "sweep" in k and k != "_meta":
            print(k[:60], v)


if __name__ == "__main__":
    main(*sys.argv[1:8])
