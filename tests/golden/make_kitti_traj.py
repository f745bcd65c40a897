"""Pack the KITTI-00 ground-truth trajectory shipped with the reference (kitti_ground_truth_tum/00.txt, TUM
format: t tx ty tz qx qy qz qw, camera frame) into tests/golden/kitti00_gt.npz (data only) for the C3 replay
workload: the synthetic scans are generated at these poses.
Usage: python tests/golden/make_kitti_traj.py /root/reference/kitti_ground_truth_tum/00.txt"""
import os
import sys

import numpy as np

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/kitti_ground_truth_tum/00.txt"
tum = np.loadtxt(src, dtype=np.float64)
assert tum.ndim == 2 and tum.shape[1] == 8
np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "kitti00_gt.npz"), tum=tum)
print(tum.shape)
