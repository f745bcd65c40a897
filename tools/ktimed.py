"""Per-kernel durations of a rocprofv3 kernel trace over the timed steps only: each kernel's first `skip` share of its
dispatches (the bench's warm-up steps) is dropped, so that the average compares with the bench line's in-kernel stamps.
   tools/ktimed.py run_kernel_trace.csv WARMUP STEPS"""
import collections
import csv
import sys

path, warm, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
by = collections.defaultdict(list)
for r in sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"])):
    by[r["Kernel_Name"].split("(")[0].replace("void ", "")].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"timed steps only: the first {warm}/{warm + steps} of each kernel's dispatches dropped")
for name, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    k = len(d) * warm // (warm + steps)
    t = sorted(d[k:])
    if not t:
        continue
    print(f"{name[:44]:44s} {len(t):7d} avg {sum(t) / len(t):8.2f} us  median {t[len(t) // 2]:8.2f} us  per step {sum(t) / steps:8.2f} us")
