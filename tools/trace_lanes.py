"""Timeline of a few scans of a rocprofv3 kernel trace (C3): every kernel with its queue, start and end relative to the
scan's k_align_init (us), then per-queue busy time per scan.  Usage: trace_lanes.py run_kernel_trace.csv [first] [count]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = int(sys.argv[2]) if len(sys.argv) > 2 else 200
count = int(sys.argv[3]) if len(sys.argv) > 3 else 3
starts = [i for i, r in enumerate(rows) if "k_align_init" in r["Kernel_Name"]]
busy = collections.defaultdict(float)
for s in range(first, min(first + count, len(starts) - 1)):
    t0 = int(rows[starts[s]]["Start_Timestamp"])
    print(f"--- scan {s}")
    for r in rows[starts[s]:starts[s + 1]]:
        a, b = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
        q = r.get("Queue_Id", "?")
        busy[q] += b - a
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ndt::", "")
        print(f"  q{q:>3s} {a:8.1f} {b:8.1f} {b - a:7.1f}  {name[:40]}")
    print(f"  next scan at {(int(rows[starts[s + 1]]['Start_Timestamp']) - t0) / 1e3:.1f} us")
print("busy per queue per scan (us):", {q: round(v / count, 1) for q, v in busy.items()})
