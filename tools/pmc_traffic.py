"""HBM traffic per launch of the derivative-pass kernel from the tools/pmc.sh counter passes.

Per /opt/skills/guides/MI355X_MICROARCH.md (HBM [CDNA4]): rocprofv3 FETCH_SIZE / WRITE_SIZE are KiB per
dispatch from the L2 memory-side request counters; on gfx950 FETCH_SIZE reports half the bytes of wide
coalesced reads, so it is doubled; WRITE_SIZE is taken as is.  Infinity-Cache hits are counted, not excluded.
The pass mixes 16 B coalesced point loads, 4 B grid probes and 64 B record gathers, so the absolute value is
uncalibrated for this pattern (ratios between variants of the kernel are exact).
Usage: python tools/pmc_traffic.py gpurun_out/pmc profiles/pmc_traffic.json ["source note"]
"""
import json
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json"
summary = json.loads(subprocess.check_output([sys.executable, "tools/pmc_summary.py", src]))
name = next(k for k in summary if "k_pass_lead" in k or "k_pass_direct" in k)
c = summary[name]
fetch = c["FETCH_SIZE"] * 1024.0
write = c["WRITE_SIZE"] * 1024.0
out = {
    "kernel": name,
    "fetch_size_bytes_raw": fetch,
    "write_size_bytes": write,
    "hbm_bytes_per_launch": 2.0 * fetch + write,
    "l2_hit_rate": (c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])) if "TCC_HIT_sum" in c else None,
    "correction": "2 x FETCH_SIZE (gfx950 half-counted wide reads) + WRITE_SIZE; KiB -> bytes",
    "counters": c,
}
if len(sys.argv) > 3:
    out["source"] = sys.argv[3]
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "counters"}, indent=1))
