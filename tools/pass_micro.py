"""Micro-benchmark of one derivative pass (k_pass_direct through the ndt_derivatives test hook) at the workload's guess
pose, repeated: kernel time under rocprofv3 (tools/gpu_libab.sh-style A/B of variant libraries), result printed so that
variants can be checked for equal arithmetic.  python tools/pass_micro.py [c2|c5] [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
import xchu_slam_amd as xa  # noqa: E402
from xchu_slam_amd import synth  # noqa: E402

wl_name = sys.argv[1] if len(sys.argv) > 1 else "c5"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
wl = bench.WORKLOADS[wl_name]
p = bench.make_pool(0, 1, wl)[0]
ndt = xa.NormalDistributionsTransform(device=0)
ndt.setNeighborhoodSearchMethod(xa.DIRECT7)
ndt.setResolution(wl["resolution"])
if os.environ.get("MICRO_PPT"):
    ndt.set_pass_options(points_per_thread=int(os.environ["MICRO_PPT"]))
G = np.asarray(p.guess, np.float64)
src = p.source
if os.environ.get("MICRO_SORT", "1") == "1":
    # the align visits clouds of >= 256 Ki points in target-cell order of the guess-transformed point (k_src_keys)
    xt = (src[:, :3].astype(np.float64) @ G[:3, :3].T + G[:3, 3]).astype(np.float32)
    inv = np.float32(1.0 / wl["resolution"])
    ijk = np.floor(xt * inv).astype(np.int64)
    ijk -= ijk.min(0)
    dims = ijk.max(0) + 1
    key = ijk[:, 0] + dims[0] * (ijk[:, 1] + dims[1] * ijk[:, 2])
    src = src[np.argsort(key, kind="stable")]
ndt.setInputTarget(p.target)
ndt.setInputSource(src)
ndt.computeDerivatives(np.zeros(6), np.eye(4), True)
# a ctx sizes its dense cell grid from the previous build's extent: the second build is the one an align stream sees
ndt.setInputTarget(p.target)
print("grid", {k: v for k, v in ndt.grid_info().items() if k in ("dense", "n_cloud", "cells")})
rpy = [np.arctan2(G[2, 1], G[2, 2]), -np.arcsin(np.clip(G[2, 0], -1, 1)), np.arctan2(G[1, 0], G[0, 0])]
x = np.array([G[0, 3], G[1, 3], G[2, 3], *rpy])
out = ndt.computeDerivatives(x, p.guess, True)
t0 = time.perf_counter()
for _ in range(reps):
    out = ndt.computeDerivatives(x, p.guess, True)
dt = (time.perf_counter() - t0) / reps
score, g, H, pairs = out
print(f"{wl_name}: N={len(p.source)} pairs={pairs} score={score:.17g} |g|={np.abs(g).sum():.17g} |H|={np.abs(H).sum():.17g} "
      f"host {dt * 1e6:.1f} us/pass")
