"""Align time per call with a fixed source size vs sizes that change every call (odom_node's filtered scans): the
cost of re-capturing the pass chain when the size leaves its geometry bucket.  Usage: python tools/vary_n.py"""
import time, sys, os
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tests"))
import xchu_slam_amd as xa
from helpers import small_pair
pair = small_pair(seed=3)
g = xa.NormalDistributionsTransform()
g.setResolution(1.0)
g.setTransformationEpsilon(0.01)
g.setMaximumIterations(30)
g.setInputTarget(pair.target)
src = np.asarray(pair.source, np.float32)
print("source points", len(src))
for mode in ("fixed", "varying", "fixed", "varying"):
    ts = []
    for k in range(60):
        n = len(src) - (0 if mode == "fixed" else (k % 7) * 13)
        g.setInputSource(src[:n])
        t0 = time.perf_counter()
        g.align(pair.guess, want_output=False)
        ts.append(time.perf_counter() - t0)
    print(mode, "median align ms", round(1e3 * float(np.median(ts[10:])), 3), "passes", g.result()["n_passes"])
