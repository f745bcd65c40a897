"""CPU checks of the odom_node replay restatement (tests/odom_restate.py) and of the KITTI-00 replay inputs."""
import math

import numpy as np
import pytest

import odom_restate as R
from xchu_slam_amd import synth


@pytest.fixture(scope="module")
def tum():
    import os
    from conftest import ROOT
    return np.load(os.path.join(ROOT, "tests", "golden", "kitti00_gt.npz"))["tum"]


def test_kitti_fixture_shape(tum):
    # kitti_ground_truth_tum/00.txt: 4541 poses, t tx ty tz qx qy qz qw
    assert tum.shape == (4541, 8)
    q = tum[:, 4:8]
    assert np.allclose(np.linalg.norm(q, axis=1), 1.0, atol=1e-6)


def test_pose_matrix_round_trip():
    rng = np.random.default_rng(0)
    for _ in range(200):
        p = np.concatenate([rng.uniform(-300, 300, 3), rng.uniform(-math.pi, math.pi, 1), rng.uniform(-1.4, 1.4, 1),
                            rng.uniform(-math.pi, math.pi, 1)])
        p = p[[0, 1, 2, 3, 4, 5]]
        m = R.pose_to_matrix(p)
        # Z*Y*X Euler (common.h:64-71) agrees with synth.pose_matrix (numpy) to float precision
        assert np.allclose(m, synth.pose_matrix(*p), atol=1e-4)
        q = R.matrix_to_pose(m)
        assert np.allclose(q[:3], p[:3], atol=1e-4)
        d = (q[3:] - p[3:] + math.pi) % (2 * math.pi) - math.pi
        assert np.all(np.abs(d) < 2e-6 / max(1e-3, math.cos(p[4])))


def test_kitti_poses_are_z_up(tum):
    P = synth.kitti_poses(tum, count=50)
    # the vehicle drives along its own x axis (camera z): displacement mostly along R[:, 0]
    d = P[10, :3, 3] - P[0, :3, 3]
    assert d[0] * P[0, 0, 0] + d[1] * P[0, 1, 0] > 0.9 * np.linalg.norm(d)
    assert np.allclose(P[:, 2, 3], 1.73)
    for k in range(len(P)):
        assert np.allclose(P[k, :3, :3] @ P[k, :3, :3].T, np.eye(3), atol=1e-6)


def test_restated_replay_tracks_ground_truth(tum, oracle):
    world, poses, scans = synth.make_sequence(tum, 10, 8000, seed=3)
    o = R.OdomRestatement(ndt_resolution=1.0, num_threads=4)
    P0 = np.linalg.inv(poses[0])
    recs = [o.process(s) for s in scans]
    o.close()
    for k, r in enumerate(recs):
        gt = P0 @ poses[k]
        assert np.linalg.norm(r["t_localizer"][:3, 3] - gt[:3, 3]) < 0.15, k
    assert recs[0]["keyframe"] is False and all(r["keyframe"] for r in recs[1:])
    # localmap reset after max_submap_size (5 m) of keyframe travel (odom_node.cpp:352-356)
    assert any(r["localmap_reset"] for r in recs)
