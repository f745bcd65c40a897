"""One step's kernel timeline from a rocprofv3 kernel trace: every kernel of the step in start order with its offset from
the step's first kernel, its duration and the idle gap before it, then the step's busy / idle split (median step).  A
step starts at each dispatch of START (default k_minmax: the target build of a registration).
   python tools/step_timeline.py run_kernel_trace.csv [START] [--queue Q]"""
import collections
import csv
import sys

path = sys.argv[1]
start_name = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "k_minmax"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
steps, cur = [], None
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if start_name in name:
        cur = []
        steps.append(cur)
    if cur is not None:
        cur.append((name, s, e))
steps = [st for st in steps if st]
if not steps:
    sys.exit("no step found")
spans = sorted(((st[-1][2] - st[0][1]) / 1e3, i) for i, st in enumerate(steps))
mid = steps[spans[len(spans) // 2][1]]
t0 = mid[0][1]
prev_end = t0
busy = 0.0
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
print(f"{len(steps)} steps; median step span {spans[len(spans) // 2][0]:.1f} us; its kernels:")
for name, s, e in mid:
    gap = max(0.0, (s - prev_end) / 1e3)
    dur = (e - s) / 1e3
    busy += dur
    a = agg[name[:44]]
    a[0] += 1; a[1] += dur; a[2] += gap
    prev_end = max(prev_end, e)
for name, (n, dur, gap) in sorted(agg.items(), key=lambda kv: -(kv[1][1] + kv[1][2])):
    print(f"  {name:44s} x{n:3d}  busy {dur:8.2f} us  idle before {gap:7.2f} us")
span = (mid[-1][2] - t0) / 1e3
print(f"step span {span:.1f} us: kernels {busy:.1f} us, idle {span - busy:.1f} us")
# the build part: kernels before the first pass kernel
first_pass = next((i for i, k in enumerate(mid) if "k_pass" in k[0]), len(mid))
if first_pass:
    b_span = (mid[first_pass - 1][2] - t0) / 1e3
    b_busy = sum((e - s) / 1e3 for _, s, e in mid[:first_pass])
    print(f"before the first pass kernel: span {b_span:.1f} us, kernels {b_busy:.1f} us, {first_pass} launches")
