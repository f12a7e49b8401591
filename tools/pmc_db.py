"""Per-kernel sums of rocprofv3 --pmc counters from its SQLite output
(<dir>/<name>_results.db; one row per dispatch x counter x dimension).
Usage: python tools/pmc_db.py <db> [kernel-substring ...]"""
import collections
import sqlite3
import sys


def per_kernel(db):
    c = sqlite3.connect(db)
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for name, counter, value, did in c.execute(
            "select kernel_name, counter_name, value, dispatch_id from counters_collection"):
        acc[name][counter] += value
        disp[name].add(did)
    return acc, disp


if __name__ == "__main__":
    acc, disp = per_kernel(sys.argv[1])
    keys = sys.argv[2:]
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        if keys and not any(s in k for s in keys):
            continue
        n = len(disp[k])
        print(k[:70], f"dispatches={n}")
        for cn, val in sorted(v.items()):
            print(f"    {cn:24s} {val / n:16.4g} per dispatch")
