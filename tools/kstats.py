"""Summarise a rocprofv3 kernel_stats.csv: per-kernel calls, average and total time per step."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.3f} ms, per step {tot / 1e3 / steps:.2f} us")
for r in rows:
    name = r["Name"].split("(")[0].replace("void ", "")
    print(f"{name[:44]:44s} {int(r['Calls']):7d} avg {float(r['AverageNs']) / 1e3:8.2f} us  per step {float(r['TotalDurationNs']) / 1e3 / steps:8.2f} us")
