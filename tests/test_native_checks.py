"""Host checks of device-side restatements that have a scalar twin (compiled with g++ -ffp-contract=off, run here).

* angle_table_entry (one lane per entry of computeAngleDerivatives' tables, ndt_omp_impl.hpp:286-398) vs
  angle_table_row: bit-exact on random angles (tests/native/angle_table_check.cpp).
"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_angle_table_entries_bit_exact(tmp_path):
    exe = tmp_path / "atc"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(HERE, "native", "angle_table_check.cpp")], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatched: 0" in out.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_packed_pair_math_bit_exact(tmp_path):
    """pair_pk (the derivative pass's pair arithmetic as packed f32 pairs, ndt_pair.h) == pair_f32 (one f32 operation per
    reference operation, ndt_omp_impl.hpp:491-548) on 400 k random pairs, with and without the Hessian."""
    exe = tmp_path / "ppc"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(HERE, "native", "pair_pk_check.cpp")], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatched: 0" in out.stdout

def _quadmath_ok(tmp_path) -> bool:
    src = tmp_path / "q.cpp"
    src.write_text("#include <quadmath.h>\nint main(){ return (int)expq((__float128)0); }\n")
    return subprocess.run(["g++", str(src), "-lquadmath", "-o", str(tmp_path / "q")], capture_output=True).returncode == 0


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_libm_restatements_correctly_rounded(tmp_path):
    """exp_dr == RN_f32(RN_f64(e^x)) (updateDerivatives' (float)exp((double)x) with glibc 2.23's correctly rounded exp,
    libndt_omp.so 0x424a4-0x424bc) and sinf_dr / cosf_dr == the correctly rounded f32 sin / cos (the model of the
    binary's sincosf), against libquadmath wherever this host's double libm cannot decide: every 61st f32 bit pattern plus
    every 7th pattern of [-2, 0] (exp) and [-0.1, 0.1] (sin / cos).  Also asserts that the oracle's own expressions
    ((float)std::exp((double)x), (float)std::sin((double)x)) give the same values.  Exhaustive run (stride 1): see
    DESIGN.md section 2."""
    if not _quadmath_ok(tmp_path):
        pytest.skip("libquadmath not available")
    exe = tmp_path / "libm"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fopenmp", "-o", str(exe),
                    os.path.join(HERE, "native", "libm_check.cpp"), "-lquadmath"], check=True)
    out = subprocess.run([str(exe), "61"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatched: 0" in out.stdout
    for line in out.stdout.splitlines():
        if "host-libm-rounded differs" in line:
            assert "host-libm-rounded differs 0 " in line, line


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_pair_orders_match_binary_sse(tmp_path):
    """pair_f32 / pair_pk (the device's per-pair f32 arithmetic) and mat3_mul_f (convertTransform's rotation products)
    against a transcription of the shipped libndt_omp.so's instruction sequences into SSE intrinsics (updateDerivatives
    0x422a0 with its Eigen product callees, computePointDerivatives 0x4b650, Transform::rotate 0x3da70; read as text,
    never run): every accumulated value equal on 300 k random pairs (tests/native/sse_order_check.cpp)."""
    exe = tmp_path / "sse"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-msse2", "-o", str(exe),
                    os.path.join(HERE, "native", "sse_order_check.cpp")], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatched: 0" in out.stdout
