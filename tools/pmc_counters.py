"""Summarise a rocprofv3 --pmc counter_collection.csv into per-kernel
averages per dispatch (small JSON), for kernels whose name contains one of
the given substrings:  python tools/pmc_counters.py <csv> <out.json> k1 [k2 ...]"""
import collections
import csv
import json
import sys


def main(path, out, keys):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if not any(s in k for s in keys):
            continue
        name = k.split("(")[0]
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name][r["Counter_Name"]].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    res = {}
    for name, cs in acc.items():
        res[name] = {c: {"per_dispatch": v / max(len(disp[name][c]), 1), "dispatches": len(disp[name][c])}
                     for c, v in cs.items()}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
