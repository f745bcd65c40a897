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

def test_libm_restatements_match_glibc(tmp_path):
    """exp_f, sinf_r, cosf_r (the device's restatements of glibc's expf / sinf / cosf, ndt_libm.h) == this host's glibc, the
    functions the reference calls (ndt_omp_impl.hpp:507; Eigen::AngleAxisf in convertTransform, ndt_omp.h:210-229), bit
    for bit: every 61st f32 bit pattern, all of [-2, 0] for expf and all of [-0.1, 0.1] for sinf / cosf."""
    exe = tmp_path / "libm"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fopenmp", "-o", str(exe),
                    os.path.join(HERE, "native", "libm_check.cpp")], check=True)
    out = subprocess.run([str(exe), "61"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatched: 0" in out.stdout

