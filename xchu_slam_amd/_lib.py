"""ctypes binding of libndt_hip.so (the C-ABI declared in include/ndt_hip.h).

The product path has exactly one implementation: the HIP library.  There is no CPU fallback; if the
shared object is missing or fails to load this module raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# NDT_HIP_LIB selects a profiling build (libndt_hip_dbg.so, `make VARIANT=dbg`); default: the product library
LIB_PATH = os.path.join(_HERE, os.environ.get("NDT_HIP_LIB", "libndt_hip.so"))

NDT_OK, NDT_EINVAL, NDT_ENOTARGET, NDT_ENOSOURCE, NDT_EOVERFLOW, NDT_EDEVICE, NDT_ENOMEM = range(7)
KDTREE, DIRECT26, DIRECT7, DIRECT1 = range(4)

STATUS_NAMES = {
    NDT_OK: "NDT_OK", NDT_EINVAL: "NDT_EINVAL", NDT_ENOTARGET: "NDT_ENOTARGET", NDT_ENOSOURCE: "NDT_ENOSOURCE",
    NDT_EOVERFLOW: "NDT_EOVERFLOW", NDT_EDEVICE: "NDT_EDEVICE", NDT_ENOMEM: "NDT_ENOMEM",
}


class NdtParams(C.Structure):
    _fields_ = [
        ("resolution", C.c_float),
        ("step_size", C.c_double),
        ("trans_eps", C.c_double),
        ("outlier_ratio", C.c_double),
        ("max_iter", C.c_int),
        ("search", C.c_int),
        ("min_points_per_voxel", C.c_int),
        ("min_covar_eigvalue_mult", C.c_double),
        ("precision_mode", C.c_int),
        ("device", C.c_int),
    ]


class NdtResult(C.Structure):
    _fields_ = [
        ("final_tf", C.c_float * 16),
        ("nr_iterations", C.c_int),
        ("converged", C.c_int),
        ("trans_probability", C.c_double),
        ("score", C.c_double),
        ("n_passes", C.c_int),
        ("n_pairs", C.c_longlong),
        ("solver_fallbacks", C.c_int),
    ]


class NdtPassRecord(C.Structure):
    _fields_ = [
        ("kind", C.c_int),
        ("newton_iter", C.c_int),
        ("x", C.c_double * 6),
        ("score", C.c_double),
        ("g", C.c_double * 6),
        ("H", C.c_double * 36),
        ("pairs", C.c_longlong),
    ]


class NdtPairDesc(C.Structure):
    _fields_ = [
        ("d_target_xyz4", C.c_void_p),
        ("n_target", C.c_size_t),
        ("d_source_xyz4", C.c_void_p),
        ("n_source", C.c_size_t),
        ("guess", C.c_float * 16),
    ]


class FilterParams(C.Structure):
    _fields_ = [
        ("leaf", C.c_float),
        ("r_min", C.c_double),
        ("r_max", C.c_double),
        ("mean_k", C.c_int),
        ("stddev_mul", C.c_double),
        ("outlier_method", C.c_int),
        ("ror_radius", C.c_double),
        ("ror_min_neighbors", C.c_int),
    ]


class OdomParams(C.Structure):
    _fields_ = [
        ("ndt_resolution", C.c_float),
        ("ndt_step_size", C.c_double),
        ("ndt_trans_eps", C.c_double),
        ("ndt_max_iter", C.c_int),
        ("min_add_scan_shift", C.c_double),
        ("max_submap_size", C.c_double),
        ("init_pose", C.c_double * 6),
        ("localmap_leaf", C.c_float),
        ("search", C.c_int),
        ("compute_fitness", C.c_int),
        ("device", C.c_int),
        ("method_type", C.c_int),
        ("incremental_voxel_update", C.c_int),
    ]


class Pose6D(C.Structure):
    _fields_ = [(k, C.c_double) for k in ("x", "y", "z", "roll", "pitch", "yaw")]


class OdomResult(C.Structure):
    _fields_ = [
        ("init_guess", C.c_float * 16),
        ("t_localizer", C.c_float * 16),
        ("t_base_link", C.c_float * 16),
        ("guess_pose", Pose6D),
        ("localizer_pose", Pose6D),
        ("current_pose", Pose6D),
        ("diff_pose", Pose6D),
        ("fitness_score", C.c_double),
        ("shift_dis", C.c_double),
        ("localmap_size", C.c_double),
        ("has_converged", C.c_int),
        ("final_num_iteration", C.c_int),
        ("keyframe", C.c_int),
        ("localmap_reset", C.c_int),
        ("n_localmap", C.c_longlong),
        ("n_tmp_map", C.c_longlong),
        ("n_target", C.c_longlong),
        ("n_appended", C.c_longlong),
        ("n_passes", C.c_int),
        ("n_pairs", C.c_longlong),
        ("ms_align", C.c_double),
        ("ms_fitness", C.c_double),
        ("ms_map", C.c_double),
        ("ms_total", C.c_double),
    ]


# name -> (restype, argtypes); the full exported surface of include/ndt_hip.h and include/ndt_odom.h
_P = C.c_void_p
_FP = C.POINTER(C.c_float)
_DP = C.POINTER(C.c_double)
SIGNATURES = {
    "ndt_default_params": (C.c_int, [C.POINTER(NdtParams)]),
    "ndt_create": (C.c_int, [C.POINTER(NdtParams), C.POINTER(_P)]),
    "ndt_set_params": (C.c_int, [_P, C.POINTER(NdtParams)]),
    "ndt_set_target": (C.c_int, [_P, _FP, C.c_size_t, C.c_size_t, C.c_int]),
    "ndt_set_target_device": (C.c_int, [_P, _P, C.c_size_t, C.c_int]),
    "ndt_set_target_append_device": (C.c_int, [_P, _P, C.c_size_t, C.c_size_t, C.c_int, _P]),
    "ndt_update_target": (C.c_int, [_P, _FP, C.c_size_t, C.c_size_t]),
    "ndt_update_target_device": (C.c_int, [_P, _P, C.c_size_t]),
    "ndt_set_source": (C.c_int, [_P, _FP, C.c_size_t, C.c_size_t]),
    "ndt_set_source_device": (C.c_int, [_P, _P, C.c_size_t]),
    "ndt_align": (C.c_int, [_P, _FP, C.POINTER(NdtResult)]),
    "ndt_align_async": (C.c_int, [_P, _FP]),
    "ndt_align_wait": (C.c_int, [_P, C.POINTER(NdtResult)]),
    "ndt_get_output": (C.c_int, [_P, _FP, C.c_size_t]),
    "ndt_get_history": (C.c_int, [_P, C.POINTER(NdtPassRecord), C.c_int, C.POINTER(C.c_int)]),
    "ndt_derivatives": (C.c_int, [_P, _DP, _FP, C.c_int, _DP, _DP, _DP, C.POINTER(C.c_longlong)]),
    "ndt_hessian_radius": (C.c_int, [_P, _DP, _FP, _DP, C.POINTER(C.c_longlong)]),
    "ndt_calculate_score": (C.c_int, [_P, _FP, _DP]),
    "ndt_fitness_score": (C.c_int, [_P, _FP, C.c_double, _DP, _FP]),
    "ndt_fitness_score_async": (C.c_int, [_P, _FP, C.c_double]),
    "ndt_fitness_score_result": (C.c_int, [_P, _DP]),
    "ndt_fitness_index_async": (C.c_int, [_P]),
    "ndt_fitness_score_async_cloud": (C.c_int, [_P, _FP, C.c_double, _P, C.c_size_t]),
    "ndt_fitness_score_async_aligned": (C.c_int, [_P, C.c_double, _P, C.c_size_t]),
    "ndt_keyframe_insert_async": (C.c_int, [_P, _FP, _P, C.c_size_t, C.c_float, _P, C.c_size_t, _P, C.c_size_t]),
    "ndt_keyframe_insert_result": (C.c_int, [_P, C.POINTER(C.c_size_t)]),
    "ndt_side_lanes_mark": (C.c_int, [_P]),
    "ndt_grid_info": (C.c_int, [_P, C.POINTER(C.c_int)]),
    "ndt_grid_leaves": (C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int), _DP, _DP, _FP, C.c_int, C.POINTER(C.c_int)]),
    "ndt_align_batch": (C.c_int, [_P, C.POINTER(NdtPairDesc), C.c_int, C.POINTER(NdtResult)]),
    "ndt_voxel_downsample": (C.c_int, [_P, _FP, C.c_size_t, C.c_size_t, C.c_int, C.c_float, _FP, C.c_size_t,
                                       C.POINTER(C.c_size_t)]),
    "ndt_transform_device": (C.c_int, [_P, _FP, _P, C.c_size_t, _P]),
    "ndt_voxel_downsample_device": (C.c_int, [_P, _P, C.c_size_t, C.c_float, _P, C.POINTER(C.c_size_t)]),
    "ndt_filter_default_params": (C.c_int, [C.POINTER(FilterParams)]),
    "ndt_filter_scan": (C.c_int, [_P, C.POINTER(FilterParams), _FP, C.c_size_t, C.c_size_t, C.c_int, _FP, C.c_size_t,
                                  C.POINTER(C.c_size_t)]),
    "ndt_filter_scan_device": (C.c_int, [_P, C.POINTER(FilterParams), _P, C.c_size_t, _P, C.POINTER(C.c_size_t)]),
    "ndt_filter_last_stats": (C.c_int, [_P, _FP, C.c_size_t, C.POINTER(C.c_size_t), _DP]),
    "ndt_memcpy_d2d": (C.c_int, [_P, _P, _P, C.c_size_t]),
    "ndt_device_alloc": (C.c_int, [_P, C.c_size_t, C.POINTER(_P)]),
    "ndt_device_free": (C.c_int, [_P, _P]),
    "ndt_memcpy_h2d": (C.c_int, [_P, _P, _P, C.c_size_t]),
    "ndt_memcpy_d2h": (C.c_int, [_P, _P, _P, C.c_size_t]),
    "ndt_synchronize": (C.c_int, [_P]),
    "ndt_last_timings": (C.c_int, [_P, _DP, _DP, _DP, _DP]),
    "ndt_pass_phases": (C.c_int, [_P, _DP]),
    "ndt_set_profiling": (C.c_int, [_P, C.c_int]),
    "ndt_set_pass_options": (C.c_int, [_P, C.c_int, C.c_int, C.c_int]),
    "ndt_set_build_options": (C.c_int, [_P, C.c_int, C.c_int]),
    "ndt_build_stats": (C.c_int, [_P, C.POINTER(C.c_longlong)]),
    "ndt_last_error": (C.c_char_p, [_P]),
    "ndt_abi_version": (C.c_int, []),
    "ndt_destroy": (None, [_P]),
    # include/ndt_odom.h (odom_node replay driver)
    "ndt_odom_default_params": (C.c_int, [C.POINTER(OdomParams)]),
    "ndt_odom_create": (C.c_int, [C.POINTER(OdomParams), C.POINTER(_P)]),
    "ndt_odom_process": (C.c_int, [_P, _FP, C.c_size_t, C.c_size_t, C.c_double, C.POINTER(OdomResult)]),
    "ndt_odom_process_device": (C.c_int, [_P, _P, C.c_size_t, C.c_double, C.POINTER(OdomResult)]),
    "ndt_odom_process_batch_device": (C.c_int, [_P, C.POINTER(_P), C.POINTER(C.c_size_t), _DP, C.c_int, C.POINTER(OdomResult)]),
    "ndt_odom_registration": (_P, [_P]),
    "ndt_odom_get_cloud": (C.c_int, [_P, C.c_int, _FP, C.c_size_t, C.POINTER(C.c_size_t)]),
    "ndt_odom_last_error": (C.c_char_p, [_P]),
    "ndt_odom_destroy": (None, [_P]),
}

_lib = None
# struct layouts this binding mirrors (include/ndt_hip.h NDT_HIP_ABI_VERSION); load() refuses a library built otherwise
ABI_VERSION = 2


def load() -> C.CDLL:
    """Load libndt_hip.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                           f"or `make -C xchu_slam_amd/csrc`")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            # an older variant library selected with NDT_HIP_LIB for an A/B run may lack a newer entry point; the
            # product library must export every one (tests/test_abi.py)
            if os.path.basename(LIB_PATH) == "libndt_hip.so":
                raise
            continue
        fn.restype = res
        fn.argtypes = args
    if lib.ndt_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH}: ABI version {lib.ndt_abi_version()}, this binding mirrors {ABI_VERSION}")
    _lib = lib
    return lib


class NdtError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


def check(status: int, ctx=None):
    if status != NDT_OK:
        msg = ""
        if ctx is not None:
            raw = load().ndt_last_error(ctx)
            msg = raw.decode() if raw else ""
        raise NdtError(status, msg)
