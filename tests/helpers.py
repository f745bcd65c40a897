"""Shared workload builders for the tests (small sizes so the CPU oracle finishes in seconds)."""
import math

import numpy as np

from xchu_slam_amd import synth


def small_pair(seed=3, half=40.0, density=6.0, n_source=4000, max_range=30.0, perturb=(0.3, 0.3, 0.05, 0.5, 0.5, 1.0)):
    w = synth.make_world(seed, half=half)
    return synth.make_pair(w, density, n_source, seed=seed + 11, max_range=max_range, perturb=perturb)


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b))))


def pose_err(T, Tref):
    d = np.linalg.inv(Tref.astype(np.float64)) @ T.astype(np.float64)
    ang = math.degrees(math.acos(max(-1.0, min(1.0, (np.trace(d[:3, :3]) - 1) / 2))))
    return float(np.linalg.norm(d[:3, 3])), ang
