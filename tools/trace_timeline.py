"""Print a kernel + copy timeline (start_us gap_us dur_us name) from a
rocprofv3 csv output directory (--kernel-trace --memory-copy-trace
--output-format csv): the last `--last` entries, times relative to the first
of them.  Used for the TwoStep host-gap analysis (profiles/r4m, r4z)."""
import argparse
import csv
import glob
import os


def rows(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "")))
    return sorted(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=40)
    a = ap.parse_args()
    ev = rows(a.dir)[-a.last:]
    t0 = ev[0][0]
    prev_end = ev[0][0]
    busy = 0
    for s, e, n in ev:
        print(f"{(s - t0) / 1e3:9.1f} {max(0, s - prev_end) / 1e3:7.1f} {(e - s) / 1e3:7.1f} {n}")
        busy += e - s
        prev_end = max(prev_end, e)
    print(f"# span {(prev_end - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
