"""GPU parity at the bench's own configuration, every pass (BASELINE configs[1], [3], [4]).

tests/test_gpu_fullsize.py stops the Newton loop after 3-4 iterations; these cases run exactly what bench.py times:
max_iter 30, trans_eps 0 (computeTransformation, ndt_omp_impl.hpp:114-159: the loop ends when nr_iterations > max_iter,
i.e. 1 + 32 derivative passes), DIRECT7, step 0.1 — on the bench's own pairs — and compare EVERY pass with the CPU
oracle run on the host's threads:

* C2: the bench's 120k-point scans vs their ~1.84M-point / ~195k-voxel localmaps at res 1.0 (pairs 0 and 1 of
  bench.make_pool), leading-tail chain (k_pass_lead, one tile per CU) and the last-workgroup-tail chain
  (k_pass_direct, ndt_align_batch's kernel) both;
* C4: one device-generated pair of the batched replay (synth_pairs.hip, pair index 7) registered through
  ndt_align_batch at 30 iterations;
* C5: the 1M-point scan vs ~1.8M voxels at res 0.5 at 10 iterations (13 passes; the oracle needs ~1 s per pass there).

Bars (tests/helpers.py): every pass's pair count exact, every per-pass parameter vector within X_TOL = 1e-12 (north
star: 1e-4 m / 1e-4 rad per iteration), the same pass kinds / Newton iterations / iteration count / convergence flag,
final transform within TF_TOL = 1e-6, and every pass's score within 1e-9 relative, gradient and Hessian within 1e-9 of
their largest entries over the align.
"""
import os
import sys

import numpy as np
import pytest

from helpers import TF_TOL, X_TOL, pose_err, rel_err

pytestmark = pytest.mark.gpu

xa = pytest.importorskip("xchu_slam_amd")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (the bench's own workload generators and MAX_ITER)

NT = max(1, min(16, os.cpu_count() or 1))  # oracle threads: the GPU box's CPU share
BENCH_PRM = dict(step_size=0.1, trans_eps=0.0, max_iter=bench.MAX_ITER, search=xa.DIRECT7)


def _device(target, source, resolution, lead_tail=True, **prm):
    g = xa.NormalDistributionsTransform()
    g._params.resolution = resolution
    for k, v in prm.items():
        setattr(g._params, k, v)
    g._push()
    g.set_pass_options(lead_tail=lead_tail)
    g.setInputTarget(target)
    g.setInputSource(source)
    return g


def _oracle(oracle, target, source, resolution, **prm):
    o = oracle.OracleNDT(num_threads=NT, resolution=resolution, **prm)
    o.set_target(target)
    o.set_source(source)
    return o


def _every_pass(ho, hg, n_expect=None):
    """Per-pass parity of two histories: kind, Newton iteration, parameter vector, pair count, score / g / H."""
    assert len(ho) == len(hg), (len(ho), len(hg))
    if n_expect is not None:
        assert len(ho) == n_expect, len(ho)
    worst = 0.0
    # gradient / Hessian within 1e-9 of their largest entries over the align (near convergence g itself is a sum of
    # cancelling terms: its size says nothing about the f64 summation-order noise)
    g_scale = max(float(np.max(np.abs(a["g"]))) for a in ho)
    h_scale = max(float(np.max(np.abs(a["H"]))) for a in ho)
    for k, (a, b) in enumerate(zip(ho, hg)):
        assert a["kind"] == b["kind"] and a["newton_iter"] == b["newton_iter"], k
        dx = float(np.max(np.abs(a["x"] - b["x"])))
        worst = max(worst, dx)
        assert dx < X_TOL, (k, dx)
        assert a["pairs"] == b["pairs"], (k, a["pairs"], b["pairs"])
        assert abs(a["score"] - b["score"]) <= 1e-9 * abs(a["score"]), k
        assert float(np.max(np.abs(b["g"] - a["g"]))) <= 1e-9 * g_scale, k
        assert float(np.max(np.abs(b["H"] - a["H"]))) <= 1e-9 * h_scale, k
    return worst


@pytest.mark.timeout(900)
@pytest.mark.parametrize("pair_index", [0, 1])
def test_c2_bench_align_every_pass(oracle, pair_index):
    """C2 as the bench times it: 33 passes, every pass vs the oracle (leading-tail chain: the bench's kernel)."""
    wl = bench.WORKLOADS["c2"]
    pair = bench.make_pool(0, pair_index + 1, wl)[pair_index]
    o = _oracle(oracle, pair.target, pair.source, wl["resolution"], **BENCH_PRM)
    g = _device(pair.target, pair.source, wl["resolution"], **BENCH_PRM)
    ro = o.align(pair.guess)
    g.align(pair.guess, want_output=False)
    rg = g.result()
    # max_iter 30, eps 0: nr_iterations > max_iter ends the loop after 32 Newton steps
    assert ro["nr_iterations"] == 32 and ro["n_passes"] == 33
    assert rg["nr_iterations"] == ro["nr_iterations"] and rg["converged"] == ro["converged"]
    assert rg["n_passes"] == ro["n_passes"] and rg["n_pairs"] == ro["n_pairs"]
    hg = g.history()
    worst = _every_pass(o.history(), hg, n_expect=33)
    assert np.max(np.abs(rg["final_tf"] - ro["final_tf"])) < TF_TOL
    t_err, r_err = pose_err(rg["final_tf"], pair.true_pose)
    assert t_err < 0.5 and r_err < 1.0, (t_err, r_err)
    print(f"C2 pair {pair_index}: 33 passes, worst per-pass |dx| {worst:.2e}, pose err {t_err:.3f} m {r_err:.3f} deg")
    # the same align through the last-workgroup-tail chain (ndt_align_batch's kernel): bitwise the same records
    g.set_pass_options(lead_tail=False)
    g.align(pair.guess, want_output=False)
    rd = g.result()
    hd = g.history()
    assert np.array_equal(rd["final_tf"], rg["final_tf"]) and rd["n_pairs"] == rg["n_pairs"]
    assert len(hd) == len(hg)
    for a, b in zip(hg, hd):
        assert np.array_equal(a["x"], b["x"]) and a["pairs"] == b["pairs"]
    _every_pass(o.history(), hd, n_expect=33)
    o.close()
    g.close()


@pytest.mark.timeout(900)
def test_c4_bench_pair_30_iterations(oracle):
    """C4: a device-generated pair of the batched replay (pair index 7), 30 iterations through ndt_align_batch — the
    final result and pair total vs the oracle on the same points, and every pass through a single align of the same
    pair on the same ctx (ndt_align_batch's per-pair records are bit-identical to single aligns)."""
    import ctypes as C
    from xchu_slam_amd import synth
    wl = bench.WORKLOADS["c4"]
    g = xa.NormalDistributionsTransform()
    g.setResolution(wl["resolution"])
    g.setTransformationEpsilon(0.0)
    g.setMaximumIterations(bench.MAX_ITER)
    lib = g._lib
    d_world = g.device_upload(np.zeros(65536, np.float32))
    spec = synth.c4_pair_spec(7, half=wl["half"], density=wl["density"], n_source=wl["n_source"], max_range=wl["max_range"])
    buf = g.device_upload(np.zeros((spec.n_target + spec.n_source, 4), np.float32))
    dt, ds = buf, buf + 16 * spec.n_target
    synth.generate_pair_device(spec, 0, d_world, dt, ds)
    t = np.empty((spec.n_target, 4), np.float32)
    s = np.empty((spec.n_source, 4), np.float32)
    lib.ndt_memcpy_d2h(g.ctx, t.ctypes.data_as(C.c_void_p), C.c_void_p(dt), t.nbytes)
    lib.ndt_memcpy_d2h(g.ctx, s.ctypes.data_as(C.c_void_p), C.c_void_p(ds), s.nbytes)
    rb = g.align_batch([(dt, spec.n_target, ds, spec.n_source, spec.guess)])[0]
    o = _oracle(oracle, t[:, :3].copy(), s[:, :3].copy(), wl["resolution"], **BENCH_PRM)
    ro = o.align(spec.guess)
    assert ro["n_passes"] == 33
    assert rb["nr_iterations"] == ro["nr_iterations"] and rb["converged"] == ro["converged"]
    assert rb["n_passes"] == ro["n_passes"] and rb["n_pairs"] == ro["n_pairs"]
    assert np.max(np.abs(rb["final_tf"] - ro["final_tf"])) < TF_TOL
    # every pass: the same pair aligned once more on the ctx (last-workgroup tails, as inside the batch)
    g.set_pass_options(lead_tail=False)
    g.setInputTargetDevice(dt, spec.n_target)
    g.setInputSourceDevice(ds, spec.n_source)
    g.align(spec.guess, want_output=False)
    rg = g.result()
    assert np.array_equal(rg["final_tf"], rb["final_tf"]) and rg["n_pairs"] == rb["n_pairs"]
    _every_pass(o.history(), g.history(), n_expect=33)
    t_err, _ = pose_err(rb["final_tf"], spec.true_pose)
    assert t_err < 0.5
    o.close()
    g.close()


@pytest.mark.timeout(1200)
def test_c5_bench_align_10_iterations(oracle):
    """C5 (dense stress, res 0.5): the bench's 1M-point scan (visited in target-cell order, two points per thread,
    multi-tile passes) vs ~1.8M voxels, 10 iterations = 13 passes, every pass vs the oracle."""
    wl = bench.WORKLOADS["c5"]
    pair = bench.make_pool(0, 1, wl)[0]
    prm = dict(BENCH_PRM, max_iter=10)
    o = _oracle(oracle, pair.target, pair.source, wl["resolution"], **prm)
    g = _device(pair.target, pair.source, wl["resolution"], **prm)
    ro = o.align(pair.guess)
    g.align(pair.guess, want_output=False)
    rg = g.result()
    assert ro["n_passes"] == 13
    assert rg["nr_iterations"] == ro["nr_iterations"] and rg["converged"] == ro["converged"]
    assert rg["n_pairs"] == ro["n_pairs"]
    worst = _every_pass(o.history(), g.history(), n_expect=13)
    assert np.max(np.abs(rg["final_tf"] - ro["final_tf"])) < TF_TOL
    t_err, _ = pose_err(rg["final_tf"], pair.true_pose)
    assert t_err < 0.5
    print(f"C5: 13 passes, worst per-pass |dx| {worst:.2e}, pose err {t_err:.3f} m")
    o.close()
    g.close()
