"""ctypes wrapper of the CPU oracle (oracle/_build/libndt_oracle.so) — TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker / CPU baseline.
Parity status of the oracle: UNPINNED (see oracle/ndt_oracle.cpp header and DESIGN.md).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")


class OrcParams(C.Structure):
    _fields_ = [("resolution", C.c_float), ("step_size", C.c_double), ("trans_eps", C.c_double), ("outlier_ratio", C.c_double),
                ("max_iter", C.c_int), ("search", C.c_int), ("min_points_per_voxel", C.c_int),
                ("min_covar_eigvalue_mult", C.c_double), ("num_threads", C.c_int), ("precision_mode", C.c_int),
                ("exp_mode", C.c_int)]


class OrcResult(C.Structure):
    _fields_ = [("final_tf", C.c_float * 16), ("nr_iterations", C.c_int), ("converged", C.c_int),
                ("trans_probability", C.c_double), ("score", C.c_double), ("n_passes", C.c_int), ("n_pairs_total", C.c_longlong)]


class OrcPassRecord(C.Structure):
    _fields_ = [("kind", C.c_int), ("newton_iter", C.c_int), ("x", C.c_double * 6), ("score", C.c_double), ("g", C.c_double * 6),
                ("H", C.c_double * 36), ("pairs", C.c_longlong)]


_libs: dict[str, C.CDLL] = {}


def build_oracle():
    subprocess.run(["make", "-C", ORACLE_DIR, "-s"], check=True)


def load(variant: str = "") -> C.CDLL:
    name = f"libndt_oracle{variant}.so"
    if name in _libs:
        return _libs[name]
    path = os.path.join(ORACLE_DIR, "_build", name)
    if not os.path.exists(path):
        build_oracle()
    lib = C.CDLL(path)
    P, FP, DP = C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_double)
    sig = {
        "orc_create": (P, []), "orc_destroy": (None, [P]), "orc_default_params": (None, [C.POINTER(OrcParams)]),
        "orc_set_params": (None, [P, C.POINTER(OrcParams)]),
        "orc_set_target": (C.c_int, [P, FP, C.c_size_t, C.c_size_t, C.c_int]),
        "orc_set_source": (C.c_int, [P, FP, C.c_size_t, C.c_size_t]),
        "orc_update_target": (C.c_int, [P, FP, C.c_size_t, C.c_size_t]),
        "orc_aw_eigen3": (None, [DP, DP, DP]),
        "orc_align": (C.c_int, [P, FP, C.POINTER(OrcResult), FP]),
        "orc_history_size": (C.c_int, [P]), "orc_history": (C.c_int, [P, C.POINTER(OrcPassRecord), C.c_int]),
        "orc_derivatives": (C.c_double, [P, DP, FP, C.c_int, DP, DP, C.POINTER(C.c_longlong)]),
        "orc_hessian_radius": (None, [P, DP, FP, DP, C.POINTER(C.c_longlong)]),
        "orc_calculate_score": (C.c_double, [P, FP]),
        "orc_convert_transform": (None, [DP, FP]), "orc_initial_p": (None, [FP, DP]),
        "orc_convert_transform_mode": (None, [DP, FP, C.c_int]),
        "orc_gauss_constants": (None, [P, DP]),
        "orc_grid_header": (None, [P, C.POINTER(C.c_int)]),
        "orc_grid_leaves": (C.c_int, [P, C.POINTER(C.c_int), C.POINTER(C.c_int), DP, DP, FP, DP, C.c_int]),
        "orc_neighbors": (C.c_int, [P, FP, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "orc_voxel_downsample": (C.c_int, [FP, C.c_size_t, C.c_size_t, C.c_int, C.c_float, FP, C.c_int]),
        "orc_filter_scan": (C.c_int, [FP, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_float, C.c_double, C.c_double, C.c_int,
                                      C.c_double, C.c_int, FP, C.c_int, FP, C.c_int, DP, C.POINTER(C.c_int), C.c_int, C.c_double,
                                      C.c_int]),
        "orc_now": (C.c_double, []),
    }
    for k, (r, a) in sig.items():
        f = getattr(lib, k)
        f.restype = r
        f.argtypes = a
    _libs[name] = lib
    return lib


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class OracleNDT:
    """CPU restatement of pclomp::NormalDistributionsTransform (same parameter names as the product wrapper)."""

    def __init__(self, variant: str = "", **params):
        self.lib = load(variant)
        self.h = self.lib.orc_create()
        self.prm = OrcParams()
        self.lib.orc_default_params(C.byref(self.prm))
        self.set(**params)
        self.n_source = 0

    def set(self, **params):
        for k, v in params.items():
            setattr(self.prm, k, v)
        self.lib.orc_set_params(self.h, C.byref(self.prm))

    def close(self):
        if self.h:
            self.lib.orc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_target(self, pts, is_dense=True):
        a = np.ascontiguousarray(pts, dtype=np.float32)
        return self.lib.orc_set_target(self.h, _fp(a), a.shape[0], a.shape[1] * 4, int(is_dense))

    def update_target(self, pts):
        """cpu::NormalDistributionsTransform::updateVoxelGrid (incremental for the ndt_cpu backend)."""
        a = np.ascontiguousarray(pts, dtype=np.float32)
        return self.lib.orc_update_target(self.h, _fp(a), a.shape[0], a.shape[1] * 4)

    def set_source(self, pts):
        a = np.ascontiguousarray(pts, dtype=np.float32)
        self.n_source = a.shape[0]
        return self.lib.orc_set_source(self.h, _fp(a), a.shape[0], a.shape[1] * 4)

    def align(self, guess=None, want_output=False):
        g = np.eye(4, dtype=np.float32) if guess is None else np.asarray(guess, np.float32)
        gc = np.ascontiguousarray(g.T).reshape(-1)
        r = OrcResult()
        out = np.empty((self.n_source, 4), np.float32) if want_output else None
        rc = self.lib.orc_align(self.h, _fp(gc), C.byref(r), _fp(out) if want_output else None)
        if rc != 0:
            raise RuntimeError("oracle align failed (no target/source)")
        res = {"final_tf": np.array(r.final_tf, np.float32).reshape(4, 4).T.copy(), "nr_iterations": r.nr_iterations,
               "converged": r.converged, "trans_probability": r.trans_probability, "score": r.score, "n_passes": r.n_passes,
               "n_pairs": r.n_pairs_total}
        if want_output:
            res["output"] = out[:, :3].copy()
        return res

    def history(self):
        n = self.lib.orc_history_size(self.h)
        recs = (OrcPassRecord * max(1, n))()
        self.lib.orc_history(self.h, recs, n)
        return [{"kind": r.kind, "newton_iter": r.newton_iter, "x": np.array(r.x[:]), "score": r.score, "g": np.array(r.g[:]),
                 "H": np.array(r.H[:]).reshape(6, 6), "pairs": r.pairs} for r in recs[:n]]

    def derivatives(self, p, T, compute_hessian=True):
        p = np.ascontiguousarray(p, np.float64)
        Tc = np.ascontiguousarray(np.asarray(T, np.float32).T).reshape(-1)
        g = np.zeros(6)
        H = np.zeros(36)
        pairs = C.c_longlong()
        s = self.lib.orc_derivatives(self.h, _dp(p), _fp(Tc), int(compute_hessian), _dp(g), _dp(H), C.byref(pairs))
        return s, g, H.reshape(6, 6), pairs.value

    def hessian_radius(self, p, T):
        p = np.ascontiguousarray(p, np.float64)
        Tc = np.ascontiguousarray(np.asarray(T, np.float32).T).reshape(-1)
        H = np.zeros(36)
        pairs = C.c_longlong()
        self.lib.orc_hessian_radius(self.h, _dp(p), _fp(Tc), _dp(H), C.byref(pairs))
        return H.reshape(6, 6), pairs.value

    def calculate_score(self, T):
        Tc = np.ascontiguousarray(np.asarray(T, np.float32).T).reshape(-1)
        return self.lib.orc_calculate_score(self.h, _fp(Tc))

    def gauss_constants(self):
        out = np.zeros(3)
        self.lib.orc_gauss_constants(self.h, _dp(out))
        return out

    def grid_header(self):
        h = (C.c_int * 15)()
        self.lib.orc_grid_header(self.h, h)
        v = list(h)
        return {"min_b": v[0:3], "max_b": v[3:6], "div_b": v[6:9], "divb_mul": v[9:12], "n_leaves": v[12], "n_cloud": v[13],
                "overflow": v[14]}

    def grid_leaves(self):
        n = self.grid_header()["n_leaves"]
        keys = np.zeros(max(n, 1), np.int32)
        npts = np.zeros(max(n, 1), np.int32)
        mean = np.zeros((max(n, 1), 3))
        icov = np.zeros((max(n, 1), 9))
        cen = np.zeros((max(n, 1), 3), np.float32)
        ev = np.zeros((max(n, 1), 3))
        self.lib.orc_grid_leaves(self.h, keys.ctypes.data_as(C.POINTER(C.c_int)), npts.ctypes.data_as(C.POINTER(C.c_int)),
                                 _dp(mean), _dp(icov), _fp(cen), _dp(ev), n)
        return {"keys": keys[:n], "npts": npts[:n], "mean": mean[:n], "icov": icov[:n].reshape(-1, 3, 3), "centroid": cen[:n],
                "evals": ev[:n]}

    def neighbors(self, pts_transformed, search):
        a = np.ones((len(pts_transformed), 4), np.float32)
        a[:, :3] = pts_transformed
        keys = np.full((len(a), 32), -1, np.int32)
        cnt = np.zeros(len(a), np.int32)
        self.lib.orc_neighbors(self.h, _fp(a), len(a), search, keys.ctypes.data_as(C.POINTER(C.c_int)),
                               cnt.ctypes.data_as(C.POINTER(C.c_int)))
        return keys, cnt


def convert_transform(x, trig_mode=1) -> np.ndarray:
    """convertTransform (ndt_omp.h:210-229); trig_mode 1 = sin / cos evaluated in double and rounded once (the model of
    the binary's sincosf), 0 = this host's glibc sinf / cosf."""
    lib = load()
    x = np.ascontiguousarray(x, np.float64)
    T = np.zeros(16, np.float32)
    lib.orc_convert_transform_mode(_dp(x), _fp(T), int(trig_mode))
    return T.reshape(4, 4).T.copy()


def initial_p(guess) -> np.ndarray:
    lib = load()
    g = np.ascontiguousarray(np.asarray(guess, np.float32).T).reshape(-1)
    p = np.zeros(6)
    lib.orc_initial_p(_fp(g), _dp(p))
    return p


def voxel_downsample(xyzi: np.ndarray, leaf: float) -> np.ndarray:
    lib = load()
    a = np.ascontiguousarray(xyzi, np.float32)
    out = np.empty((max(1, len(a)), 4), np.float32)
    n = lib.orc_voxel_downsample(_fp(a), len(a), a.shape[1] * 4, 3, float(leaf), _fp(out), len(a))
    if n < 0:
        return out[: -n].copy()
    return out[:n].copy()


def filter_scan(xyzi: np.ndarray, leaf=0.5, r_min=1.0, r_max=60.0, mean_k=30, stddev_mul=1.0, is_dense=True, brute=False,
                outlier_method=0, ror_radius=0.8, ror_min_neighbors=5):
    """filter_node front end restated (oracle/ndt_oracle.cpp orc_filter_scan): (out (K,4), distances, thr[3], n_voxel)."""
    lib = load()
    a = np.ascontiguousarray(xyzi, np.float32)
    out = np.empty((max(1, len(a)), 4), np.float32)
    dist = np.zeros(max(1, len(a)), np.float32)
    thr = np.zeros(3, np.float64)
    nv = C.c_int()
    k = lib.orc_filter_scan(_fp(a), len(a), a.shape[1] * 4, 3, 1 if is_dense else 0, float(leaf), float(r_min), float(r_max),
                            int(mean_k), float(stddev_mul), 1 if brute else 0, _fp(out), len(a), _fp(dist), len(a), _dp(thr),
                            C.byref(nv), int(outlier_method), float(ror_radius), int(ror_min_neighbors))
    return out[:k].copy(), dist[: nv.value].copy(), thr, nv.value


def aw_eigen3(A) -> tuple[np.ndarray, np.ndarray]:
    """cpu::SymmetricEigensolver3x3 (ndt_cpu) restated: (eigenvalues, eigenvector columns)."""
    a = np.ascontiguousarray(np.asarray(A, np.float64).T).reshape(-1)
    ev = np.zeros(3)
    V = np.zeros(9)
    load().orc_aw_eigen3(_dp(a), _dp(ev), _dp(V))
    return ev, V.reshape(3, 3).T.copy()


def now() -> float:
    return load().orc_now()
