"""Summarise tools/pmc.sh output: per-dispatch averages of every counter for the filtered kernel."""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = defaultdict(list)
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        vals[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
out = {}
for (k, c), v in sorted(vals.items()):
    out.setdefault(k, {})[c] = sum(v) / len(v)
print(json.dumps(out, indent=1))
