"""Print sweep-kernel rows of rocprofv3 *_kernel_stats.csv files:
python tools/kstats_csv.py <csv> [substring ...]"""
import csv
import sys

keys = sys.argv[2:] or ["sweep"]
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in keys):
        print(f"  {r['Name'].split('(')[0][:44]:44s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs']) / 1e3:9.1f}")
