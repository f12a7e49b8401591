"""Per-sweep span from a rocprofv3 kernel_trace.csv: the sweep kernels
(k_sweep_band x3, k_sweep_tiled, k_sweep_flat) run on three streams and
overlap, so rocprof's per-kernel averages are concurrent spans; the sweep's
duration is max(end) - min(start) over its dispatches, grouped by the k_marg
that follows each sweep.  python tools/sweep_span.py <trace.csv> <out.json>"""
import csv
import json
import sys


def main(path, out):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    spans, cur = [], []
    for r in rows:
        name = r["Kernel_Name"]
        if "k_sweep_" in name:
            cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        elif "k_marg" in name and cur:
            spans.append((max(e for _, e in cur) - min(s for s, _ in cur)) / 1e6)
            cur = []
    res = {"sweeps": len(spans), "span_ms_avg": sum(spans) / max(len(spans), 1),
           "span_ms_min": min(spans) if spans else None, "span_ms_max": max(spans) if spans else None}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
