"""Shared workload builders for the tests (small sizes so the CPU oracle finishes in seconds)."""
import math

import numpy as np

from xchu_slam_amd import synth


def small_pair(seed=3, half=40.0, density=6.0, n_source=4000, max_range=30.0, perturb=(0.3, 0.3, 0.05, 0.5, 0.5, 1.0)):
    w = synth.make_world(seed, half=half)
    return synth.make_pair(w, density, n_source, seed=seed + 11, max_range=max_range, perturb=perturb)


# Parity bars of a full align against the oracle (the device evaluates every per-pair f32 term, the transform and the
# Newton control's reductions as the shipped libndt_omp.so does, and so does the oracle, DESIGN.md §2 — only the f64
# summation order of the 43 sums differs; tools/parity_margins.py measures the margins)
X_TOL = 1e-12    # per-pass parameter vector (f64)
TF_TOL = 1e-6    # final f32 transform


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b))))


def pose_err(T, Tref):
    d = np.linalg.inv(Tref.astype(np.float64)) @ T.astype(np.float64)
    ang = math.degrees(math.acos(max(-1.0, min(1.0, (np.trace(d[:3, :3]) - 1) / 2))))
    return float(np.linalg.norm(d[:3, 3])), ang


def raw_scan(seed=21, half=90.0, n_points=40000, max_range=80.0, n_nan=50, n_outliers=200):
    """A raw HDL-64-like scan for filter_node's front end, sensor frame, (N, 4) x,y,z,intensity: LiDAR-like
    surfaces out to max_range (the 60 m crop removes some), a few non-finite points and isolated outliers in the air."""
    rng = np.random.default_rng(seed)
    w = synth.make_world(seed, half=half)
    pose = synth.pose_matrix(0.0, 0.0, 1.73, 0.0, 0.0, 0.3)
    pts = synth.sensor_scan(w, pose, n_points, seed + 1, max_range=max_range)
    out = rng.uniform(-40, 40, (n_outliers, 3)).astype(np.float32)
    out[:, 2] = rng.uniform(3, 15, n_outliers)
    cloud = np.concatenate([pts, out]).astype(np.float32)
    inten = rng.uniform(0, 1, (len(cloud), 1)).astype(np.float32)
    cloud = np.concatenate([cloud, inten], 1)
    nan_idx = rng.choice(len(cloud), n_nan, replace=False)
    cloud[nan_idx, rng.integers(0, 3, n_nan)] = np.nan
    return cloud[rng.permutation(len(cloud))]
