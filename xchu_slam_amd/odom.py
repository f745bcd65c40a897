"""Python handle on the odom_node scan-loop replay driver (include/ndt_odom.h, C++ in csrc/odom_estimate.cpp).

LidarOdom restates LidarOdom::OdomEstimate (/root/reference/xchu_mapping/src/odom_node.cpp:208-356) without ROS:
feed scans in order with `process(scan, stamp)` (host) or `process_device(ptr, n, stamp)` (HBM-resident float4);
each call returns the per-scan record (guess, t_localizer, poses, fitness, keyframe/reset flags, cloud sizes).
The loop itself is native C++; this module only marshals arrays.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import OdomParams, OdomResult, check

_POSE_KEYS = ("x", "y", "z", "roll", "pitch", "yaw")
LOCALMAP, TMP_MAP, TARGET = 0, 1, 2


def _mat(a) -> np.ndarray:
    return np.array(list(a), np.float32).reshape(4, 4).T.copy()  # column-major -> row-major


def _pose(p) -> np.ndarray:
    return np.array([getattr(p, k) for k in _POSE_KEYS])


class LidarOdom:
    """odom_node (use_omp backend, no IMU / wheel odometry) over the MI355X registration."""

    def __init__(self, device: int = 0, **params):
        self._lib = _lib.load()
        self._p = OdomParams()
        check(self._lib.ndt_odom_default_params(C.byref(self._p)))
        self._p.device = device
        for k, v in params.items():
            if k == "init_pose":
                for i in range(6):
                    self._p.init_pose[i] = float(v[i])
            else:
                setattr(self._p, k, v)
        h = C.c_void_p()
        check(self._lib.ndt_odom_create(C.byref(self._p), C.byref(h)))
        self._h = h
        self._ctx = self._lib.ndt_odom_registration(h)
        self._dev = []

    def close(self):
        if getattr(self, "_h", None):
            for p in self._dev:
                self._lib.ndt_device_free(self._ctx, C.c_void_p(p))
            self._dev = []
            self._lib.ndt_odom_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st):
        if st != _lib.NDT_OK:
            raw = self._lib.ndt_odom_last_error(self._h)
            raise _lib.NdtError(st, raw.decode() if raw else "")

    @staticmethod
    def _record(r: OdomResult) -> dict:
        return {
            "init_guess": _mat(r.init_guess), "t_localizer": _mat(r.t_localizer), "t_base_link": _mat(r.t_base_link),
            "guess_pose": _pose(r.guess_pose), "localizer_pose": _pose(r.localizer_pose),
            "current_pose": _pose(r.current_pose), "diff_pose": _pose(r.diff_pose),
            "fitness_score": r.fitness_score, "shift_dis": r.shift_dis, "localmap_size": r.localmap_size,
            "has_converged": bool(r.has_converged), "final_num_iteration": r.final_num_iteration,
            "keyframe": bool(r.keyframe), "localmap_reset": bool(r.localmap_reset),
            "n_localmap": r.n_localmap, "n_tmp_map": r.n_tmp_map, "n_target": r.n_target, "n_appended": r.n_appended,
            "n_passes": r.n_passes, "n_pairs": r.n_pairs,
            "ms_align": r.ms_align, "ms_fitness": r.ms_fitness, "ms_map": r.ms_map, "ms_total": r.ms_total,
        }

    def process(self, scan: np.ndarray, stamp: float) -> dict:
        a = np.ascontiguousarray(scan, np.float32)
        if a.ndim != 2 or a.shape[1] < 3:
            raise ValueError("scan must have shape (N, >=3)")
        r = OdomResult()
        self._check(self._lib.ndt_odom_process(self._h, a.ctypes.data_as(C.POINTER(C.c_float)), len(a), a.shape[1] * 4,
                                               float(stamp), C.byref(r)))
        return self._record(r)

    def upload(self, scan: np.ndarray) -> tuple[int, int]:
        """Copy a scan into HBM as float4 x,y,z,intensity (owned by this object); returns (device ptr, n)."""
        a = np.zeros((len(scan), 4), np.float32)
        a[:, :3] = np.asarray(scan)[:, :3]
        if np.asarray(scan).shape[1] > 3:
            a[:, 3] = np.asarray(scan)[:, 3]
        ptr = C.c_void_p()
        check(self._lib.ndt_device_alloc(self._ctx, max(a.nbytes, 16), C.byref(ptr)), self._ctx)
        check(self._lib.ndt_memcpy_h2d(self._ctx, ptr, a.ctypes.data_as(C.c_void_p), a.nbytes), self._ctx)
        self._dev.append(ptr.value)
        return ptr.value, len(a)

    def process_device(self, ptr: int, n: int, stamp: float) -> dict:
        r = OdomResult()
        self._check(self._lib.ndt_odom_process_device(self._h, C.c_void_p(ptr), n, float(stamp), C.byref(r)))
        return self._record(r)

    def process_batch_device(self, scans: list[tuple[int, int]], stamps) -> list[dict]:
        """ndt_odom_process_batch_device: the (device ptr, n) scans in order, pipelined; one record per scan."""
        k = len(scans)
        ptrs = (C.c_void_p * max(k, 1))(*[p for p, _ in scans])
        ns = (C.c_size_t * max(k, 1))(*[n for _, n in scans])
        st = (C.c_double * max(k, 1))(*[float(t) for t in stamps])
        out = (OdomResult * max(k, 1))()
        self._check(self._lib.ndt_odom_process_batch_device(self._h, ptrs, ns, st, k, out))
        return [self._record(out[i]) for i in range(k)]

    def cloud(self, which: int = LOCALMAP) -> np.ndarray:
        n = C.c_size_t()
        self._check(self._lib.ndt_odom_get_cloud(self._h, which, None, 0, C.byref(n)))
        out = np.empty((max(1, n.value), 4), np.float32)
        self._check(self._lib.ndt_odom_get_cloud(self._h, which, out.ctypes.data_as(C.POINTER(C.c_float)), n.value,
                                                 C.byref(n)))
        return out[: n.value]

    def timings(self) -> dict:
        b, a, p, y = C.c_double(), C.c_double(), C.c_double(), C.c_double()
        check(self._lib.ndt_last_timings(self._ctx, C.byref(b), C.byref(a), C.byref(p), C.byref(y)), self._ctx)
        return {"ms_build": b.value, "ms_align": a.value, "ms_pass_avg": p.value, "pass_bytes_avg": y.value}

    def set_profiling(self, on: bool):
        check(self._lib.ndt_set_profiling(self._ctx, 1 if on else 0), self._ctx)
