"""Host-side mirror of pclomp::NormalDistributionsTransform<PointXYZI, PointXYZI> backed by libndt_hip.so.

Method names, argument meaning, defaults and error behaviour follow the reference registration object
(/root/reference/xchu_mapping/include/pclomp/ndt_omp.h:70-497, ndt_omp_impl.hpp:46-164) and the
pcl::Registration surface odom_node drives (odom_node.cpp:69-80, 227-228, 277-283, 348-349):

    ndt = NormalDistributionsTransform()
    ndt.setNeighborhoodSearchMethod(DIRECT7); ndt.setTransformationEpsilon(0.01)
    ndt.setStepSize(0.1); ndt.setResolution(1.0); ndt.setMaximumIterations(30)
    ndt.setInputTarget(localmap); ndt.setInputSource(scan)
    output = ndt.align(guess)
    T = ndt.getFinalTransformation(); ndt.hasConverged(); ndt.getFinalNumIteration()

All numerics run in HIP kernels on the GPU; the Python layer only marshals arrays.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import DIRECT1, DIRECT7, DIRECT26, KDTREE, NdtPairDesc, NdtParams, NdtPassRecord, NdtResult, check

__all__ = ["NormalDistributionsTransform", "CpuNormalDistributionsTransform", "KDTREE", "DIRECT26", "DIRECT7", "DIRECT1", "as_points", "voxel_downsample"]

POINT_XYZI_DTYPE = np.dtype({"names": ["x", "y", "z", "data3", "intensity"], "formats": ["<f4"] * 5,
                             "offsets": [0, 4, 8, 12, 16], "itemsize": 32})


def as_points(cloud) -> tuple[np.ndarray, int]:
    """Return (contiguous float32 buffer, stride in bytes) for an (N,3)/(N,4) float array or a PointXYZI record array."""
    a = np.asarray(cloud)
    if a.dtype.names is not None:
        if a.dtype.itemsize < 12 or a.dtype.fields["x"][1] != 0:
            raise ValueError("structured clouds must start with float x,y,z")
        a = np.ascontiguousarray(a)
        return a.view(np.uint8).reshape(-1).view(np.float32), a.dtype.itemsize
    a = np.ascontiguousarray(a, dtype=np.float32)
    if a.ndim != 2 or a.shape[1] < 3:
        raise ValueError("point cloud must have shape (N, >=3)")
    return a, a.shape[1] * 4


def _fp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class NormalDistributionsTransform:
    """pclomp::NormalDistributionsTransform on MI355X (one HIP stream per instance, not thread-safe)."""

    def __init__(self, device: int = 0):
        self._lib = _lib.load()
        self._params = NdtParams()
        check(self._lib.ndt_default_params(C.byref(self._params)))
        self._params.device = device
        ctx = C.c_void_p()
        check(self._lib.ndt_create(C.byref(self._params), C.byref(ctx)))
        self._ctx = ctx
        self._result = NdtResult()
        self._n_source = 0
        self._has_result = False
        self.num_threads = 1

    # ------------------------------------------------------------------ lifetime
    def close(self):
        if getattr(self, "_ctx", None):
            self._lib.ndt_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def ctx(self):
        return self._ctx

    def _push(self):
        check(self._lib.ndt_set_params(self._ctx, C.byref(self._params)), self._ctx)

    # ------------------------------------------------------------------ parameters (ndt_omp.h:110-186)
    def setNumThreads(self, n: int):
        # OpenMP thread count of the CPU reference; the GPU path ignores it (kept for API compatibility)
        self.num_threads = int(n)

    def setResolution(self, resolution: float):
        self._params.resolution = float(resolution)
        self._push()

    def getResolution(self) -> float:
        return float(self._params.resolution)

    def setStepSize(self, step_size: float):
        self._params.step_size = float(step_size)
        self._push()

    def getStepSize(self) -> float:
        return float(self._params.step_size)

    def setOulierRatio(self, ratio: float):
        self._params.outlier_ratio = float(ratio)
        self._push()

    def getOulierRatio(self) -> float:
        return float(self._params.outlier_ratio)

    def setNeighborhoodSearchMethod(self, method: int):
        self._params.search = int(method)
        self._push()

    def setTransformationEpsilon(self, eps: float):
        self._params.trans_eps = float(eps)
        self._push()

    def getTransformationEpsilon(self) -> float:
        return float(self._params.trans_eps)

    def setMaximumIterations(self, n: int):
        self._params.max_iter = int(n)
        self._push()

    def getMaximumIterations(self) -> int:
        return int(self._params.max_iter)

    def setPrecisionMode(self, mode: int):
        """0 = ndt_omp (f32 per pair), 1 = pcl::NormalDistributionsTransform (f64 per pair, radius search),
        2 = cpu::NormalDistributionsTransform (ndt_cpu: its own VoxelGrid and radius search, f64 per pair)."""
        self._params.precision_mode = int(mode)
        self._push()

    def setMinPointPerVoxel(self, n: int):
        # VoxelGridCovariance::setMinPointPerVoxel (voxel_grid_covariance_omp.h:135-146): values <= 2 become 3
        self._params.min_points_per_voxel = int(n) if n > 2 else 3
        self._push()

    def params(self) -> dict:
        return {k: getattr(self._params, k) for k, _ in NdtParams._fields_}

    # ------------------------------------------------------------------ inputs
    def setInputTarget(self, cloud, is_dense: bool = True):
        buf, stride = as_points(cloud)
        n = buf.size * 4 // stride if buf.size else 0
        check(self._lib.ndt_set_target(self._ctx, _fp(buf), n, stride, int(bool(is_dense))), self._ctx)
        self._has_result = False

    def setInputTargetDevice(self, d_ptr: int, n: int, is_dense: bool = True):
        check(self._lib.ndt_set_target_device(self._ctx, C.c_void_p(d_ptr), n, int(bool(is_dense))), self._ctx)
        self._has_result = False

    def setInputTargetAppendDevice(self, d_ptr: int, n_old: int, n_new: int, is_dense: bool = True, d_new: int = 0):
        """setInputTarget of a device cloud whose first n_old points are the current target's (odom_node's growing
        localmap, odom_node.cpp:233 / 349): the same grid as setInputTargetDevice(d_ptr, n_old + n_new), built by merging
        the new points' sort into the current one when the ctx still holds it.  d_new: the new points are read there and
        stored at d_ptr's point n_old by the build."""
        check(self._lib.ndt_set_target_append_device(self._ctx, C.c_void_p(d_ptr), n_old, n_new, int(bool(is_dense)),
                                                     C.c_void_p(d_new) if d_new else None), self._ctx)
        self._has_result = False

    def updateVoxelGrid(self, cloud):
        """cpu::NormalDistributionsTransform::updateVoxelGrid (ndt_cpu/NormalDistributionsTransform.h:39,
        odom_node.cpp:344-345): the points join the target after the existing ones, the grid follows."""
        buf, stride = as_points(cloud)
        n = buf.size * 4 // stride if buf.size else 0
        check(self._lib.ndt_update_target(self._ctx, _fp(buf), n, stride), self._ctx)
        self._has_result = False

    def updateVoxelGridDevice(self, d_ptr: int, n: int):
        check(self._lib.ndt_update_target_device(self._ctx, C.c_void_p(d_ptr), n), self._ctx)
        self._has_result = False

    def setInputSource(self, cloud):
        buf, stride = as_points(cloud)
        n = buf.size * 4 // stride if buf.size else 0
        check(self._lib.ndt_set_source(self._ctx, _fp(buf), n, stride), self._ctx)
        self._n_source = n
        self._has_result = False

    def setInputSourceDevice(self, d_ptr: int, n: int):
        check(self._lib.ndt_set_source_device(self._ctx, C.c_void_p(d_ptr), n), self._ctx)
        self._n_source = n
        self._has_result = False

    # ------------------------------------------------------------------ alignment
    def align(self, guess=None, want_output: bool = True):
        """pcl::Registration::align(output, guess): returns the source transformed by the final transform."""
        g = np.eye(4, dtype=np.float32) if guess is None else np.asarray(guess, dtype=np.float32)
        if g.shape != (4, 4):
            raise ValueError("guess must be 4x4")
        colmajor = np.ascontiguousarray(g.T).reshape(-1)
        check(self._lib.ndt_align(self._ctx, _fp(colmajor), C.byref(self._result)), self._ctx)
        self._has_result = True
        if not want_output:
            return None
        out = np.empty((self._n_source, 4), dtype=np.float32)
        check(self._lib.ndt_get_output(self._ctx, _fp(out), 16), self._ctx)
        return out[:, :3].copy()

    def getFinalTransformation(self) -> np.ndarray:
        return np.array(self._result.final_tf, dtype=np.float32).reshape(4, 4).T.copy()

    def hasConverged(self) -> bool:
        return bool(self._result.converged)

    def getFinalNumIteration(self) -> int:
        return int(self._result.nr_iterations)

    def getTransformationProbability(self) -> float:
        return float(self._result.trans_probability)

    def result(self) -> dict:
        r = self._result
        return {"final_tf": self.getFinalTransformation(), "nr_iterations": r.nr_iterations, "converged": r.converged,
                "trans_probability": r.trans_probability, "score": r.score, "n_passes": r.n_passes, "n_pairs": r.n_pairs,
                "solver_fallbacks": r.solver_fallbacks}

    def history(self) -> list[dict]:
        n = C.c_int()
        check(self._lib.ndt_get_history(self._ctx, None, 0, C.byref(n)), self._ctx)
        recs = (NdtPassRecord * max(1, n.value))()
        check(self._lib.ndt_get_history(self._ctx, recs, n.value, C.byref(n)), self._ctx)
        out = []
        for i in range(n.value):
            r = recs[i]
            out.append({"kind": r.kind, "newton_iter": r.newton_iter, "x": np.array(r.x[:]), "score": r.score,
                        "g": np.array(r.g[:]), "H": np.array(r.H[:]).reshape(6, 6), "pairs": r.pairs})
        return out

    def computeDerivatives(self, p, T, compute_hessian: bool = True):
        """One computeDerivatives pass (ndt_omp_impl.hpp:175) at parameters p with point transform T (4x4)."""
        p = np.ascontiguousarray(p, dtype=np.float64)
        Tc = np.ascontiguousarray(np.asarray(T, dtype=np.float32).T).reshape(-1)
        score = C.c_double()
        g = np.zeros(6)
        H = np.zeros(36)
        pairs = C.c_longlong()
        check(self._lib.ndt_derivatives(self._ctx, _dp(p), _fp(Tc), int(compute_hessian), C.byref(score), _dp(g), _dp(H),
                                        C.byref(pairs)), self._ctx)
        return score.value, g, H.reshape(6, 6), pairs.value

    def computeHessianRadius(self, p, T):
        """computeHessian (ndt_omp_impl.hpp:550-607): radius neighbours, f64."""
        p = np.ascontiguousarray(p, dtype=np.float64)
        Tc = np.ascontiguousarray(np.asarray(T, dtype=np.float32).T).reshape(-1)
        H = np.zeros(36)
        pairs = C.c_longlong()
        check(self._lib.ndt_hessian_radius(self._ctx, _dp(p), _fp(Tc), _dp(H), C.byref(pairs)), self._ctx)
        return H.reshape(6, 6), pairs.value

    def calculateScore(self, T=None) -> float:
        """calculateScore (ndt_omp_impl.hpp:919-952) of the input source transformed by T (default: the final
        transformation of the last align).  The reference takes the already transformed cloud; transforming
        inside the device call (pcl::transformPointCloud arithmetic, f32) is the same computation."""
        if T is None:
            T = self.getFinalTransformation()
        Tc = np.ascontiguousarray(np.asarray(T, dtype=np.float32).T).reshape(-1)
        out = C.c_double()
        check(self._lib.ndt_calculate_score(self._ctx, _fp(Tc), C.byref(out)), self._ctx)
        return out.value

    def getFitnessScore(self, max_range: float = float(np.finfo(np.float64).max), T=None, return_distances: bool = False):
        """pcl::Registration::getFitnessScore (odom_node.cpp:280): mean squared nearest-neighbour distance from
        the transformed source to all target points (squared distances <= max_range, PCL's comparison);
        T defaults to the final transformation of the last align."""
        Tc = None if T is None else np.ascontiguousarray(np.asarray(T, dtype=np.float32).T).reshape(-1)
        out = C.c_double()
        d2 = np.zeros(max(self._n_source, 1), np.float32) if return_distances else None
        check(self._lib.ndt_fitness_score(self._ctx, None if Tc is None else _fp(Tc), float(max_range), C.byref(out),
                                          None if d2 is None else _fp(d2)), self._ctx)
        return (out.value, d2[: self._n_source]) if return_distances else out.value

    # ------------------------------------------------------------------ grid inspection
    def grid_info(self) -> dict:
        h = (C.c_int * 16)()
        check(self._lib.ndt_grid_info(self._ctx, h), self._ctx)
        v = list(h)
        return {"min_b": v[0:3], "max_b": v[3:6], "div_b": v[6:9], "divb_mul": v[9:12], "n_leaves": v[12],
                "n_cloud": v[13], "overflow": v[14], "n_valid": v[15]}

    def grid_leaves(self) -> dict:
        info = self.grid_info()
        n = info["n_cloud"]
        keys = np.zeros(max(n, 1), np.int32)
        npts = np.zeros(max(n, 1), np.int32)
        mean = np.zeros((max(n, 1), 3))
        icov = np.zeros((max(n, 1), 9))
        cen = np.zeros((max(n, 1), 3), np.float32)
        nout = C.c_int()
        check(self._lib.ndt_grid_leaves(self._ctx, keys.ctypes.data_as(C.POINTER(C.c_int)), npts.ctypes.data_as(C.POINTER(C.c_int)),
                                        _dp(mean), _dp(icov), _fp(cen), n, C.byref(nout)), self._ctx)
        return {"keys": keys[:n], "npts": npts[:n], "mean": mean[:n], "icov": icov[:n].reshape(-1, 3, 3), "centroid": cen[:n]}

    def timings(self) -> dict:
        b, a, p, by = C.c_double(), C.c_double(), C.c_double(), C.c_double()
        check(self._lib.ndt_last_timings(self._ctx, C.byref(b), C.byref(a), C.byref(p), C.byref(by)))
        ph = (C.c_double * 22)()
        check(self._lib.ndt_pass_phases(self._ctx, ph))
        names = ("bodies", "handoff", "reduce", "stage", "control", "tables", "drain")
        out = {"ms_build": b.value, "ms_align": a.value, "ms_pass_avg": p.value, "pass_bytes_avg": by.value,
               "pass_phases_ms": dict(zip(names, list(ph)[:7]))}
        if any(ph[7:12]):
            out["workgroup_phases_ms"] = dict(zip(("entry", "probe", "compact", "pairs", "block_reduce"), list(ph)[7:12]))
        if any(ph[12:22]):
            out["tail_phases_ms"] = dict(zip(("record", "machine", "solve_setup", "solve", "post_solve", "sincos", "rows",
                                              "writeback", "spec_solve_start", "spec_solve"), list(ph)[12:22]))
        return out

    def setProfiling(self, enable: bool):
        check(self._lib.ndt_set_profiling(self._ctx, int(bool(enable))))

    def set_pass_options(self, lead_tail: bool = True, points_per_thread: int = 2, source_order: bool = True):
        """ndt_set_pass_options: the pass-chain tuning / test hooks (include/ndt_hip.h)."""
        check(self._lib.ndt_set_pass_options(self._ctx, int(bool(lead_tail)), int(points_per_thread), int(bool(source_order))),
              self._ctx)

    def set_build_options(self, tile_tickets: bool = False, radix_passes: int = 0):
        """ndt_set_build_options: target-sort test hooks (include/ndt_hip.h)."""
        check(self._lib.ndt_set_build_options(self._ctx, int(bool(tile_tickets)), int(radix_passes)), self._ctx)

    def build_stats(self) -> dict:
        """ndt_build_stats: full / merge-extended / re-run target builds of this ctx and the sort mode in use."""
        out = (C.c_longlong * 6)()
        check(self._lib.ndt_build_stats(self._ctx, out), self._ctx)
        v = list(out)
        return {"full": v[0], "merge": v[1], "rerun": v[2], "rerun_lookback": v[3], "tile_tickets": v[4], "radix_passes": v[5]}

    # ------------------------------------------------------------------ device memory helpers
    def device_upload(self, arr: np.ndarray) -> int:
        a = np.ascontiguousarray(arr)
        ptr = C.c_void_p()
        check(self._lib.ndt_device_alloc(self._ctx, a.nbytes, C.byref(ptr)), self._ctx)
        check(self._lib.ndt_memcpy_h2d(self._ctx, ptr, a.ctypes.data_as(C.c_void_p), a.nbytes), self._ctx)
        return ptr.value

    def device_free(self, ptr: int):
        check(self._lib.ndt_device_free(self._ctx, C.c_void_p(ptr)), self._ctx)

    def align_batch(self, pairs: list[tuple[int, int, int, int, np.ndarray]]) -> list[dict]:
        """Offline batch: pairs of (d_target, n_target, d_source, n_source, guess4x4) device-resident float4 clouds."""
        descs = (NdtPairDesc * max(1, len(pairs)))()
        for i, (dt, nt, ds, ns, g) in enumerate(pairs):
            descs[i].d_target_xyz4 = dt
            descs[i].n_target = nt
            descs[i].d_source_xyz4 = ds
            descs[i].n_source = ns
            gc = np.ascontiguousarray(np.asarray(g, np.float32).T).reshape(-1)
            for k in range(16):
                descs[i].guess[k] = float(gc[k])
        res = (NdtResult * max(1, len(pairs)))()
        check(self._lib.ndt_align_batch(self._ctx, descs, len(pairs), res), self._ctx)
        out = []
        for i in range(len(pairs)):
            r = res[i]
            out.append({"final_tf": np.array(r.final_tf, np.float32).reshape(4, 4).T.copy(), "nr_iterations": r.nr_iterations,
                        "converged": r.converged, "trans_probability": r.trans_probability, "score": r.score,
                        "n_passes": r.n_passes, "n_pairs": r.n_pairs, "solver_fallbacks": r.solver_fallbacks})
        return out


class CpuNormalDistributionsTransform(NormalDistributionsTransform):
    """cpu::NormalDistributionsTransform<PointXYZI, PointXYZI> (ndt_cpu, odom_node's ndt_method_type 1 — the launch
    default, xchu_mapping.launch:17): Autoware's NDT with its own cpu::VoxelGrid (division binning, its closed-form
    3x3 eigen solver, radius neighbours over f64 centroids) and f64 per-pair math, on the same device path
    (precision_mode 2).  Method names follow ndt_cpu/NormalDistributionsTransform.h:11-111."""

    def __init__(self, device: int = 0):
        super().__init__(device)
        self._params.precision_mode = 2
        self._push()

    def setOutlierRatio(self, ratio: float):
        self.setOulierRatio(ratio)

    def getOutlierRatio(self) -> float:
        return self.getOulierRatio()


def voxel_downsample(cloud_xyzi: np.ndarray, leaf: float, device: int = 0, ndt: NormalDistributionsTransform | None = None):
    """pcl::VoxelGrid<PointXYZI> (leaf^3) on the GPU: returns (K, 4) x,y,z,intensity ordered by voxel index."""
    a = np.ascontiguousarray(cloud_xyzi, dtype=np.float32)
    if a.ndim != 2 or a.shape[1] < 4:
        raise ValueError("expected (N, 4) x,y,z,intensity")
    own = ndt is None
    if own:
        ndt = NormalDistributionsTransform(device)
    try:
        out = np.empty((max(1, a.shape[0]), 4), np.float32)
        nout = C.c_size_t()
        st = ndt._lib.ndt_voxel_downsample(ndt.ctx, _fp(a), a.shape[0], a.shape[1] * 4, 3, float(leaf), _fp(out), a.shape[0],
                                           C.byref(nout))
        if st not in (_lib.NDT_OK, _lib.NDT_EOVERFLOW):
            check(st, ndt.ctx)
        return out[: nout.value].copy()
    finally:
        if own:
            ndt.close()


def filter_scan(cloud_xyzi: np.ndarray, leaf: float = 0.5, r_min: float = 1.0, r_max: float = 60.0, mean_k: int = 30,
                stddev_mul: float = 1.0, device: int = 0, ndt: NormalDistributionsTransform | None = None, stats: bool = False,
                outlier_method: int = 0, ror_radius: float = 0.8, ror_min_neighbors: int = 5):
    """filter_node's front end on the GPU (xchu_mapping/src/filter_node.cpp:218-273): non-finite points dropped, range
    crop r_min < sqrt(x^2+y^2) < r_max, pcl::VoxelGrid(leaf), pcl::StatisticalOutlierRemoval(mean_k, stddev_mul)
    (outlier_method 0, filter_node's default) or pcl::RadiusOutlierRemoval(ror_radius, ror_min_neighbors) (outlier_method 1).
    Returns the /filtered_points cloud (K, 4) x,y,z,intensity; with stats=True also (distances, thr[3], n_voxel)."""
    a = np.ascontiguousarray(cloud_xyzi, dtype=np.float32)
    if a.ndim != 2 or a.shape[1] < 4:
        raise ValueError("expected (N, 4) x,y,z,intensity")
    own = ndt is None
    if own:
        ndt = NormalDistributionsTransform(device)
    try:
        prm = _lib.FilterParams()
        check(ndt._lib.ndt_filter_default_params(C.byref(prm)))
        prm.leaf, prm.r_min, prm.r_max, prm.mean_k, prm.stddev_mul = float(leaf), float(r_min), float(r_max), int(mean_k), float(stddev_mul)
        prm.outlier_method, prm.ror_radius, prm.ror_min_neighbors = int(outlier_method), float(ror_radius), int(ror_min_neighbors)
        out = np.empty((max(1, a.shape[0]), 4), np.float32)
        nout = C.c_size_t()
        check(ndt._lib.ndt_filter_scan(ndt.ctx, C.byref(prm), _fp(a), a.shape[0], a.shape[1] * 4, 3, _fp(out), a.shape[0],
                                       C.byref(nout)), ndt.ctx)
        res = out[: nout.value].copy()
        if not stats:
            return res
        dist = np.zeros(max(1, a.shape[0]), np.float32)
        nv = C.c_size_t()
        thr = np.zeros(3, np.float64)
        check(ndt._lib.ndt_filter_last_stats(ndt.ctx, _fp(dist), a.shape[0], C.byref(nv), thr.ctypes.data_as(C.POINTER(C.c_double))),
              ndt.ctx)
        return res, dist[: nv.value].copy(), thr, nv.value
    finally:
        if own:
            ndt.close()
