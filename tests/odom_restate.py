"""TEST INFRASTRUCTURE — CPU restatement of odom_node's scan loop, driven by the oracle registration.

Restates LidarOdom::OdomEstimate (/root/reference/xchu_mapping/src/odom_node.cpp:208-356) and the Pose6D helpers
(xchu_mapping/include/xchu_mapping/common.h:38-71) in plain Python over oracle/ (OracleNDT for
pclomp::NormalDistributionsTransform, orc_voxel_downsample for pcl::VoxelGrid).  Used only by tests/ as the checker of
the native C++ driver (csrc/odom_estimate.cpp); never imported by the product.

Third-party semantics restated here (absent from /root/reference): Eigen 3.3 AngleAxis::toRotationMatrix, the
fixed-size 3x3 product's unrolled redux (a0*b0 + (a1*b1 + a2*b2)), Quaternion-from-matrix (Shepperd), and ROS tf
LinearMath Matrix3x3::setRotation / getEulerYPR (solution 1).  Parity of these is "restated, unpinned" — no
golden vectors for them exist in the reference; the pose-to-matrix round trip is checked by property tests.
"""
from __future__ import annotations

import math

import numpy as np

import oracle_lib

POSE_KEYS = ("x", "y", "z", "roll", "pitch", "yaw")


def axis_rotation(angle: float, axis: int) -> list[list[float]]:
    """Eigen::AngleAxisd(angle, e_axis).toRotationMatrix()."""
    s, c = math.sin(angle), math.cos(angle)
    ax = [1.0 if axis == k else 0.0 for k in range(3)]
    sa = [s * a for a in ax]
    ca = [(1.0 - c) * a for a in ax]
    R = [[0.0] * 3 for _ in range(3)]
    t = ca[0] * ax[1]
    R[0][1] = t - sa[2]
    R[1][0] = t + sa[2]
    t = ca[0] * ax[2]
    R[0][2] = t + sa[1]
    R[2][0] = t - sa[1]
    t = ca[1] * ax[2]
    R[1][2] = t - sa[0]
    R[2][1] = t + sa[0]
    for k in range(3):
        R[k][k] = ca[k] * ax[k] + c
    return R


def mul3(A, B):
    return [[A[i][0] * B[0][j] + (A[i][1] * B[1][j] + A[i][2] * B[2][j]) for j in range(3)] for i in range(3)]


def pose_to_matrix(p) -> np.ndarray:
    """Pose6D2Matrix (common.h:64-71) then .cast<float>(): row-major float32 4x4."""
    x, y, z, roll, pitch, yaw = p
    R = mul3(mul3(axis_rotation(yaw, 2), axis_rotation(pitch, 1)), axis_rotation(roll, 0))
    m = np.eye(4, dtype=np.float32)
    m[:3, :3] = np.array(R, np.float64).astype(np.float32)
    m[:3, 3] = np.array([x, y, z], np.float64).astype(np.float32)
    return m


def matrix_to_pose(mf: np.ndarray) -> np.ndarray:
    """Matrix2Pose6D (common.h:51-63) of a float32 matrix (cast to double)."""
    m = [[float(mf[i, j]) for j in range(3)] for i in range(3)]
    q = [0.0, 0.0, 0.0, 0.0]  # x, y, z, w
    t = m[0][0] + (m[1][1] + m[2][2])
    if t > 0.0:
        t = math.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0] = (m[2][1] - m[1][2]) * t
        q[1] = (m[0][2] - m[2][0]) * t
        q[2] = (m[1][0] - m[0][1]) * t
    else:
        i = 0
        if m[1][1] > m[0][0]:
            i = 1
        if m[2][2] > m[i][i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = math.sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (m[k][j] - m[j][k]) * t
        q[j] = (m[j][i] + m[i][j]) * t
        q[k] = (m[k][i] + m[i][k]) * t
    d = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]
    s = 2.0 / d
    xs, ys, zs = q[0] * s, q[1] * s, q[2] * s
    wx, wy, wz = q[3] * xs, q[3] * ys, q[3] * zs
    xx, xy, xz = q[0] * xs, q[0] * ys, q[0] * zs
    yy, yz, zz = q[1] * ys, q[1] * zs, q[2] * zs
    r00, r10 = 1.0 - (yy + zz), xy + wz
    r20, r21, r22 = xz - wy, yz + wx, 1.0 - (xx + yy)
    if abs(r20) >= 1.0:
        yaw = 0.0
        pitch = math.pi / 2.0 if r20 < 0.0 else -math.pi / 2.0
        roll = math.atan2(r21, r22)
    else:
        pitch = -math.asin(r20)
        cp = math.cos(pitch)
        roll = math.atan2(r21 / cp, r22 / cp)
        yaw = math.atan2(r10 / cp, r00 / cp)
    return np.array([float(mf[0, 3]), float(mf[1, 3]), float(mf[2, 3]), roll, pitch, yaw])


def mul4(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    """Matrix4f product, column-wise left-associated sums in float32."""
    A = A.astype(np.float32)
    B = B.astype(np.float32)
    C = np.zeros((4, 4), np.float32)
    for j in range(4):
        C[:, j] = ((A[:, 0] * B[0, j] + A[:, 1] * B[1, j]) + A[:, 2] * B[2, j]) + A[:, 3] * B[3, j]
    return C


def transform_cloud(pts: np.ndarray, T: np.ndarray) -> np.ndarray:
    """pcl::transformPointCloud in float32: x' = ((m00 x + m01 y) + m02 z) + m03, intensity carried."""
    p = np.asarray(pts, np.float32)
    T = T.astype(np.float32)
    out = p.copy()
    for r in range(3):
        out[:, r] = ((T[r, 0] * p[:, 0] + T[r, 1] * p[:, 1]) + T[r, 2] * p[:, 2]) + T[r, 3]
    return out


class OdomRestatement:
    """OdomEstimate over OracleNDT with odom_node's defaults (use_omp, DIRECT7, no IMU/odom)."""

    def __init__(self, ndt_resolution=2.0, ndt_step_size=0.1, ndt_trans_eps=0.01, ndt_max_iter=30,
                 min_add_scan_shift=0.5, max_submap_size=5.0, localmap_leaf=1.0, num_threads=8, method_type=3,
                 incremental_voxel_update=False):
        # MethodType (odom_node.cpp:55-69): 0 pcl_ndt, 1 ndt_cpu, 3 ndt_omp
        self.ndt = oracle_lib.OracleNDT(resolution=ndt_resolution, step_size=ndt_step_size, trans_eps=ndt_trans_eps,
                                        max_iter=ndt_max_iter, search=2, num_threads=num_threads,
                                        precision_mode={0: 1, 1: 2, 3: 0}[method_type])
        self.incremental = method_type == 1 and incremental_voxel_update
        self.min_add_scan_shift = min_add_scan_shift
        self.max_localmap_size = max_submap_size
        self.leaf = localmap_leaf
        self.tf_l2b = np.eye(4, dtype=np.float32)  # init pose 0 (odom_node.cpp:86-94)
        self.localmap = np.zeros((0, 4), np.float32)
        self.tmp_map = np.zeros((0, 4), np.float32)
        self.pc_target = np.zeros((0, 4), np.float32)
        self.initial_scan_loaded = False
        self.n_keyframes = 0
        self.previous_pose = np.zeros(6)
        self.diff_pose = np.zeros(6)
        self.localmap_size = 0.0

    def close(self):
        self.ndt.close()

    def process(self, scan: np.ndarray) -> dict:
        scan4 = np.zeros((len(scan), 4), np.float32)
        scan4[:, :scan.shape[1] if scan.shape[1] <= 4 else 4] = scan[:, :4]
        if not self.initial_scan_loaded or self.n_keyframes == 0:            # :218-231
            tr = transform_cloud(scan4, self.tf_l2b)
            self.localmap = np.concatenate([self.localmap, tr])
            self.pc_target = np.concatenate([self.pc_target, tr])
            self.ndt.set_target(self.pc_target[:, :3])
            self.initial_scan_loaded = True
        self.pc_target = self.localmap.copy()                                 # :233
        guess = self.previous_pose + self.diff_pose                           # :234-236
        guess[4] = self.previous_pose[4]
        guess[3] = self.previous_pose[3]
        init_guess = pose_to_matrix(guess)                                    # :254
        self.ndt.set_source(scan4[:, :3])                                     # :277-283
        r = self.ndt.align(init_guess)
        t_localizer = r["final_tf"]
        t_base_link = mul4(t_localizer, self.tf_l2b)                          # :289
        transformed = transform_cloud(scan4, t_localizer)                     # :290
        current = matrix_to_pose(t_base_link)                                 # :292-296
        self.n_keyframes += 1
        self.diff_pose = current - self.previous_pose                         # :311
        shift = math.sqrt(math.pow(current[0] - self.previous_pose[0], 2.0) + math.pow(current[1] - self.previous_pose[1], 2.0))
        self.previous_pose = current.copy()
        keyframe = shift >= self.min_add_scan_shift
        appended = 0
        if keyframe:                                                          # :329-346
            self.localmap_size += shift
            ds = oracle_lib.voxel_downsample(transformed, self.leaf)
            appended = len(ds)
            self.localmap = np.concatenate([self.localmap, ds])
            self.tmp_map = np.concatenate([self.tmp_map, ds])
            if self.incremental:                                              # :343-345
                self.ndt.update_target(ds[:, :3])
            else:
                self.ndt.set_target(self.pc_target[:, :3])
        reset = False
        if self.localmap_size >= self.max_localmap_size:                      # :352-356
            self.localmap = self.tmp_map
            self.tmp_map = np.zeros((0, 4), np.float32)
            self.localmap_size = 0.0
            reset = True
        return {"init_guess": init_guess, "t_localizer": t_localizer, "t_base_link": t_base_link, "guess_pose": guess,
                "current_pose": current, "shift_dis": shift, "keyframe": keyframe, "localmap_reset": reset,
                "n_localmap": len(self.localmap), "n_tmp_map": len(self.tmp_map), "n_appended": appended,
                "final_num_iteration": r["nr_iterations"], "has_converged": bool(r["converged"])}
