"""C-ABI checks that need no GPU: the library builds/loads, exports every entry point of include/ndt_hip.h,
reports the reference defaults, and fails loudly (no CPU fallback) when no device is present."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT, gpu_available

HEADERS = [os.path.join(ROOT, "include", h) for h in ("ndt_hip.h", "ndt_odom.h")]
LIB = os.path.join(ROOT, "xchu_slam_amd", "libndt_hip.so")


def declared_symbols():
    text = "".join(open(h).read() for h in HEADERS)
    return sorted(set(re.findall(r"^\s*(?:ndt_status|void|int|const char\*|ndt_ctx\*)\s+(ndt_\w+)\s*\(", text, re.M)))


def test_header_declares_the_registration_surface():
    syms = declared_symbols()
    for s in ["ndt_create", "ndt_set_params", "ndt_set_target", "ndt_set_source", "ndt_align", "ndt_get_output",
              "ndt_align_batch", "ndt_voxel_downsample", "ndt_last_error", "ndt_destroy", "ndt_fitness_score",
              "ndt_calculate_score", "ndt_odom_create", "ndt_odom_process", "ndt_odom_process_device"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "xchu_slam_amd", "csrc")], check=True)
    lib = ctypes.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s(ndt_\w+)", out))
    assert set(declared_symbols()) <= exported


def test_abi_version_matches_header():
    """The library reports the struct-layout version of the header it was built with (layouts changed in
    place once; a caller compares ndt_abi_version() with NDT_HIP_ABI_VERSION)."""
    from xchu_slam_amd import _lib
    hdr = open(os.path.join(ROOT, "include", "ndt_hip.h")).read()
    want = int(re.search(r"#define NDT_HIP_ABI_VERSION (\d+)", hdr).group(1))
    assert _lib.load().ndt_abi_version() == want == _lib.ABI_VERSION


def test_binding_covers_header():
    from xchu_slam_amd import _lib
    assert set(declared_symbols()) == set(_lib.SIGNATURES)


def test_default_params_match_reference_ctor():
    from xchu_slam_amd import _lib
    lib = _lib.load()
    p = _lib.NdtParams()
    assert lib.ndt_default_params(ctypes.byref(p)) == 0
    # pclomp ctor (ndt_omp_impl.hpp:46-69) and VGC ctor (voxel_grid_covariance_omp.h:202-217)
    assert p.resolution == 1.0 and p.step_size == 0.1 and p.trans_eps == 0.1 and p.outlier_ratio == 0.55
    assert p.max_iter == 35 and p.search == _lib.DIRECT7 and p.min_points_per_voxel == 6
    assert p.min_covar_eigvalue_mult == 0.01 and p.precision_mode == 0


def test_struct_layouts(tmp_path):
    """Every ctypes mirror has the C header's size and field offsets (compiled with gcc against include/)."""
    import subprocess
    from xchu_slam_amd import _lib
    structs = {"ndt_params": _lib.NdtParams, "ndt_result": _lib.NdtResult, "ndt_pass_record": _lib.NdtPassRecord,
               "ndt_pair_desc": _lib.NdtPairDesc}
    src = ["#include <stdio.h>", "#include <stddef.h>", '#include "ndt_hip.h"', "int main(void) {"]
    for cname, py in structs.items():
        src.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            src.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    src.append("return 0; }")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(py, f).offset, (cname, f)


@pytest.mark.skipif(gpu_available(), reason="checks the no-device error path")
def test_no_device_fails_loudly():
    from xchu_slam_amd import _lib
    import xchu_slam_amd as xa
    lib = _lib.load()
    ctx = ctypes.c_void_p()
    assert lib.ndt_create(None, ctypes.byref(ctx)) == _lib.NDT_EDEVICE
    with pytest.raises(_lib.NdtError):
        xa.NormalDistributionsTransform()


def test_null_argument_errors():
    from xchu_slam_amd import _lib
    lib = _lib.load()
    assert lib.ndt_create(None, None) == _lib.NDT_EINVAL
    assert lib.ndt_default_params(None) == _lib.NDT_EINVAL
    assert lib.ndt_align(None, None, None) == _lib.NDT_EINVAL
    assert lib.ndt_last_error(None) == b"null ctx"


def test_product_never_touches_the_oracle():
    pkg = os.path.join(ROOT, "xchu_slam_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                text = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in text.lower(), f


def test_odom_defaults_match_param_initial():
    """ndt_odom_default_params = LidarOdom::ParamInitial defaults (odom_node.cpp:42-49, 86-98)."""
    from xchu_slam_amd import _lib
    lib = _lib.load()
    p = _lib.OdomParams()
    assert lib.ndt_odom_default_params(ctypes.byref(p)) == 0
    assert p.ndt_resolution == 2.0 and p.ndt_step_size == 0.1 and p.ndt_trans_eps == 0.01 and p.ndt_max_iter == 30
    assert p.min_add_scan_shift == 0.5 and p.max_submap_size == 5.0 and list(p.init_pose) == [0.0] * 6
    assert p.localmap_leaf == 1.0 and p.search == _lib.DIRECT7 and p.compute_fitness == 1
    assert ctypes.sizeof(_lib.OdomResult) == 3 * 64 + 4 * 48 + 3 * 8 + 4 * 4 + 4 * 8 + 8 + 8 + 4 * 8


@pytest.mark.skipif(gpu_available(), reason="checks the no-device error path")
def test_odom_no_device_fails_loudly():
    from xchu_slam_amd import _lib
    import xchu_slam_amd as xa
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.ndt_odom_create(None, ctypes.byref(h)) == _lib.NDT_EDEVICE
    assert lib.ndt_odom_create(None, None) == _lib.NDT_EINVAL
    assert lib.ndt_odom_last_error(None) == b"null odom"
    with pytest.raises(_lib.NdtError):
        xa.LidarOdom()
