"""rocprofv3 --kernel-trace SQLite output (<dir>/<name>_results.db) -> the
kernel_stats.csv columns rocprofv3 --stats writes in CSV mode.
Usage: python tools/kstats_db.py <db> <out.csv>"""
import collections
import csv
import math
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    d = collections.defaultdict(list)
    for name, dur in c.execute("select name, duration from kernels"):
        d[name].append(float(dur))
    tot_all = sum(sum(v) for v in d.values()) or 1.0
    rows = []
    for name, v in d.items():
        n, t = len(v), sum(v)
        mean = t / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in v) / n)
        rows.append([name, n, int(t), f"{mean:.6f}", f"{100.0 * t / tot_all:.2f}", int(min(v)), int(max(v)), f"{sd:.6f}"])
    rows.sort(key=lambda r: -r[2])
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        w.writerows(rows)


if __name__ == "__main__":
    main(*sys.argv[1:3])
