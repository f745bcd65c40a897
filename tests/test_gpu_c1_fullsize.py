"""pcl_ndt mode at C1 size (BASELINE configs[0]): a raw 120 000-point scan at KITTI-00 ground-truth
pose 50 registered against a localmap of the 10 keyframe scans at poses 0, 5, ..., 45, each 120 000 points,
downsampled at 1.0 m (pcl::VoxelGrid, odom_node.cpp:334-335) and moved into the map frame by its ground-truth pose; the
guess is the true pose perturbed by (0.3 m, 0.3 m, 0.05 m, 0.5 deg, 0.5 deg, 1.0 deg).  Same synthetic world and scan
generator as the C3 replay (bench.py c3_world / synth.sensor_scan).

Backend: precision_mode 1 = pcl::NormalDistributionsTransform (radius neighbours over the voxel centroids, f64 per pair,
serial in PCL), res 1.0, step 0.1, eps 0.01, max_iter 3 (the oracle's serial f64 radius passes are the slow part).
Per pass: the parameter vector within X_TOL = 1e-12 of the oracle's (north star 1e-4 m / 1e-4 rad), the pass kinds and
Newton indices equal, exactly the oracle's radius-pair count; iteration count, convergence and the final transform
(TF_TOL = 1e-6) as the oracle.
"""
import math
import os

import numpy as np
import pytest

from conftest import ROOT
from helpers import TF_TOL, X_TOL

pytestmark = pytest.mark.gpu

N_POINTS = 120_000


def make_c1_pair():
    """(target, source, true pose, guess) of the C1 configuration."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    import oracle_lib
    from xchu_slam_amd import synth
    tum = np.load(os.path.join(ROOT, "tests", "golden", "kitti00_gt.npz"))["tum"]
    poses = synth.kitti_poses(tum)
    world = bench.c3_world(tum, 0)
    P0 = np.linalg.inv(poses[0])
    parts = []
    for k in range(0, 50, 5):
        s = synth.sensor_scan(world, poses[k], N_POINTS, 7919 * (k + 1))
        T = P0 @ poses[k]
        m = (s.astype(np.float64) @ T[:3, :3].T + T[:3, 3]).astype(np.float32)
        parts.append(oracle_lib.voxel_downsample(m, 1.0)[:, :3])
    target = np.concatenate(parts).astype(np.float32)
    source = synth.sensor_scan(world, poses[50], N_POINTS, 7919 * 51).astype(np.float32)
    true = P0 @ poses[50]
    rng = np.random.default_rng(1)
    sgn = rng.choice([-1.0, 1.0], 6)
    d = [0.3 * sgn[0], 0.3 * sgn[1], 0.05 * sgn[2], math.radians(0.5) * sgn[3], math.radians(0.5) * sgn[4],
         math.radians(1.0) * sgn[5]]
    guess = (true @ synth.pose_matrix(*d)).astype(np.float32)
    return target, source, true, guess


@pytest.fixture(scope="module")
def c1_pair():
    return make_c1_pair()


@pytest.mark.parametrize("mode", [1, 2], ids=["pcl_ndt", "ndt_cpu"])
def test_pcl_ndt_c1_size(c1_pair, oracle, mode):
    """mode 1: pcl_ndt; mode 2: ndt_cpu (odom_node's launch default, ndt_method_type 1: cpu::VoxelGrid binning and radius
    search, parity unpinned beyond the restatement) — the same bars at C1 size."""
    import xchu_slam_amd as xa
    target, source, true, guess = c1_pair
    assert len(source) == N_POINTS and len(target) > 100_000
    prm = dict(resolution=1.0, step_size=0.1, trans_eps=0.01, max_iter=3, search=xa.DIRECT7, precision_mode=mode)
    o = oracle.OracleNDT(num_threads=1, **prm)
    o.set_target(target)
    o.set_source(source)
    ro = o.align(guess)
    g = xa.NormalDistributionsTransform()
    for k, v in prm.items():
        setattr(g._params, k, v)
    g._push()
    g.setInputTarget(target)
    g.setInputSource(source)
    g.align(guess, want_output=False)
    rg = g.result()
    ho, hg = o.history(), g.history()
    assert rg["nr_iterations"] == ro["nr_iterations"] and rg["converged"] == ro["converged"]
    assert len(ho) == len(hg) >= 3
    assert ho[0]["pairs"] == hg[0]["pairs"] and ho[0]["pairs"] > N_POINTS
    worst = 0.0
    for a, b in zip(ho, hg):
        assert a["kind"] == b["kind"] and a["newton_iter"] == b["newton_iter"]
        worst = max(worst, float(np.max(np.abs(a["x"] - b["x"]))))
        assert a["pairs"] == b["pairs"], (a["pairs"], b["pairs"])
    assert worst < X_TOL, worst
    assert np.max(np.abs(rg["final_tf"] - ro["final_tf"])) < TF_TOL
    d = np.linalg.inv(true) @ rg["final_tf"].astype(np.float64)
    assert np.linalg.norm(d[:3, 3]) < 0.3
    print(f"C1 mode {mode}: M={len(target)} N={len(source)} passes={len(hg)} pairs[0]={hg[0]['pairs']} worst |dx|={worst:.2e}")
