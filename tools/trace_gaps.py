"""Gaps between consecutive kernels of a rocprofv3 kernel trace, grouped by the pass index inside an align."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
gap_at = collections.defaultdict(list)
k, prev = 0, None
for r in rows:
    n = r["Kernel_Name"]
    if "k_align_init" in n:
        k = 0
    if "k_pass_" in n:
        k += 1
        gap_at[k].append((int(r["Start_Timestamp"]) - prev) / 1e3)
    prev = int(r["End_Timestamp"])
for k in sorted(gap_at):
    g = sorted(gap_at[k])
    print(f"pass {k:3d} n {len(g):4d} median gap {g[len(g) // 2]:7.2f} us  max {g[-1]:7.2f}")
