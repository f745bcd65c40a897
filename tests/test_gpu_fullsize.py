"""GPU parity at the BASELINE configs' full sizes against the CPU oracle run with the host's
threads.  The oracle's Newton loop is bounded (max_iter 3-4, trans_eps 0) so that each case finishes in tens of seconds;
the device runs exactly the same code path as in the 30-iteration bench (multi-tile radix sort, > 512 partial blocks,
res-0.5 key widths, the source visited in target-cell order for >= 256 Ki points, the batched multi-stream replay).

Bars (same as tests/test_gpu_parity.py): voxel grid keys / counts / means / centroids bit-exact, inverse covariances
<= 1e-12 relative; every pass's pair count exact; every per-pass parameter vector <= X_TOL = 1e-12 (north star: 1e-4 m /
1e-4 rad); identical iteration counts and convergence flags; final transform <= TF_TOL = 1e-6.
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
import bench  # noqa: E402  (the bench's own workload generators)

NT = max(1, min(16, os.cpu_count() or 1))  # oracle threads: the GPU box's CPU share


def _grid_matches(o, g):
    oh, gh = o.grid_header(), g.grid_info()
    for k in ("min_b", "max_b", "div_b", "divb_mul", "n_leaves", "n_cloud", "overflow"):
        assert oh[k] == gh[k], k
    ol, gl = o.grid_leaves(), g.grid_leaves()
    sel = (ol["npts"] >= 6) | (ol["npts"] == -1)
    for k in ("keys", "npts", "mean", "centroid"):
        assert np.array_equal(ol[k][sel], gl[k]), k
    valid = gl["npts"] > 0
    assert rel_err(gl["icov"][valid], ol["icov"][sel][valid]) < 1e-12
    return int(valid.sum())


def _objs(oracle, target, source, **prm):
    o = oracle.OracleNDT(num_threads=NT, **prm)
    o.set_target(target)
    o.set_source(source)
    g = xa.NormalDistributionsTransform()
    for k, v in prm.items():
        setattr(g._params, k, v)
    g._push()
    g.setInputTarget(target)
    g.setInputSource(source)
    return o, g


def _align_parity(o, g, guess, true_pose, t_tol=0.2):
    ro = o.align(guess)
    g.align(guess, want_output=False)
    rg = g.result()
    ho, hg = o.history(), g.history()
    assert rg["nr_iterations"] == ro["nr_iterations"]
    assert rg["converged"] == ro["converged"]
    assert len(ho) == len(hg)
    assert ho[0]["pairs"] == hg[0]["pairs"] and ho[0]["pairs"] > 0
    for a, b in zip(ho, hg):
        assert a["kind"] == b["kind"] and a["newton_iter"] == b["newton_iter"]
        assert np.max(np.abs(a["x"] - b["x"])) < X_TOL
        assert a["pairs"] == b["pairs"]
    assert np.max(np.abs(rg["final_tf"] - ro["final_tf"])) < TF_TOL
    t_err, _ = pose_err(rg["final_tf"], true_pose)
    assert t_err < t_tol
    return ho, hg


@pytest.mark.timeout(600)
def test_c2_full_size(oracle):
    """C2 (BASELINE configs[1]): the bench's own 120k-point scan vs 1.84M-point / ~195k-voxel localmap at res 1.0,
    DIRECT7 — grid bit-exact, one pass at the guess exact in P and 1e-9 in score/g/H, a 4-iteration align per pass."""
    pair = bench.make_pool(0, 1, bench.WORKLOADS["c2"])[0]
    prm = dict(resolution=1.0, step_size=0.1, trans_eps=0.0, max_iter=4, search=xa.DIRECT7)
    o, g = _objs(oracle, pair.target, pair.source, **prm)
    assert _grid_matches(o, g) > 150_000
    p = oracle.initial_p(pair.guess)
    T = pair.guess.astype(np.float32)
    so, go, Ho, Po = o.derivatives(p, T, True)
    sg, gg, Hg, Pg = g.computeDerivatives(p, T, True)
    assert Po == Pg and Po > 3 * len(pair.source)
    assert abs(so - sg) <= 1e-9 * abs(so) and rel_err(gg, go) < 1e-9 and rel_err(Hg, Ho) < 1e-9
    _align_parity(o, g, pair.guess, pair.true_pose, t_tol=0.5)
    o.close()
    g.close()


@pytest.mark.timeout(600)
def test_c2_target_multitile_lead_chain(oracle):
    """The C2 target with a 240k-point source (the bench scan and a jittered copy of it): above the one-tile leading-tail
    kernel's 196 608 points (256 CUs x 768), below the 262 144-point leading-tail limit — the 512-thread leading-tail
    kernel with its tile loop, per pass against the oracle (3 iterations)."""
    pair = bench.make_pool(0, 1, bench.WORKLOADS["c2"])[0]
    rng = np.random.default_rng(17)
    src2 = pair.source.copy()
    src2[:, :3] += rng.normal(0.0, 0.02, (len(src2), 3)).astype(np.float32)
    source = np.concatenate([pair.source, src2]).astype(np.float32)
    assert 196_608 < len(source) < 262_144
    prm = dict(resolution=1.0, step_size=0.1, trans_eps=0.0, max_iter=3, search=xa.DIRECT7)
    o, g = _objs(oracle, pair.target, source, **prm)
    _align_parity(o, g, pair.guess, pair.true_pose, t_tol=0.5)
    o.close()
    g.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("search", ["DIRECT26", "DIRECT1", "KDTREE"])
def test_c2_full_size_other_searches(oracle, search):
    """C2 at full size with ndt_omp's other neighbourhood searches (ndt_omp_impl.hpp:212-231): DIRECT26
    (getAllNeighborCellIndices, centre cell excluded), DIRECT1 (own voxel) and KDTREE (radiusSearch over the voxel
    centroids, voxel_grid_covariance_omp.h:470-499) — one pass at the guess exact in P and 1e-9 in score/g/H, a 3-iteration
    align per pass."""
    pair = bench.make_pool(0, 1, bench.WORKLOADS["c2"])[0]
    prm = dict(resolution=1.0, step_size=0.1, trans_eps=0.0, max_iter=3, search=getattr(xa, search))
    o, g = _objs(oracle, pair.target, pair.source, **prm)
    p = oracle.initial_p(pair.guess)
    T = pair.guess.astype(np.float32)
    so, go, Ho, Po = o.derivatives(p, T, True)
    sg, gg, Hg, Pg = g.computeDerivatives(p, T, True)
    assert Po == Pg and Po > len(pair.source) // 4
    assert abs(so - sg) <= 1e-9 * abs(so) and rel_err(gg, go) < 1e-9 and rel_err(Hg, Ho) < 1e-9
    # parity per pass; the pose after 3 steps of <= 0.1 m is only checked for sanity (DIRECT26 has no centre cell)
    _align_parity(o, g, pair.guess, pair.true_pose, t_tol=2.0)
    o.close()
    g.close()


@pytest.mark.timeout(900)
def test_c5_full_size_res05(oracle):
    """C5 (BASELINE configs[4]) at full size: the bench's 1M-point scan vs ~2M voxels of a ~18M-point map at res 0.5
    (dense-grid lookup, res-0.5 key widths, source in target-cell order) — grid bit-exact, 3-iteration align per pass."""
    pair = bench.make_pool(0, 1, bench.WORKLOADS["c5"])[0]
    prm = dict(resolution=0.5, step_size=0.1, trans_eps=0.0, max_iter=3, search=xa.DIRECT7)
    o, g = _objs(oracle, pair.target, pair.source, **prm)
    assert _grid_matches(o, g) > 1_500_000
    _align_parity(o, g, pair.guess, pair.true_pose, t_tol=0.5)
    o.close()
    g.close()


@pytest.mark.timeout(900)
def test_c5_full_size_direct1_pass(oracle):
    """C5's 1M-point scan through the DIRECT1 pass (two points per thread, packed pair words at this size: the
    489-point tiles leave the second point slot of the upper threads empty) — one full pass per pose vs the oracle."""
    pair = bench.make_pool(0, 1, bench.WORKLOADS["c5"])[0]
    prm = dict(resolution=0.5, step_size=0.1, trans_eps=0.0, max_iter=3, search=xa.DIRECT1)
    o, g = _objs(oracle, pair.target, pair.source, **prm)
    for pose in (pair.guess, pair.true_pose):
        p = oracle.initial_p(pose)
        T = pose.astype(np.float32)
        so, go, Ho, Po = o.derivatives(p, T, True)
        sg, gg, Hg, Pg = g.computeDerivatives(p, T, True)
        assert Po == Pg and Po > len(pair.source) // 4
        assert abs(so - sg) <= 1e-9 * abs(so) and rel_err(gg, go) < 1e-9 and rel_err(Hg, Ho) < 1e-9
    o.close()
    g.close()


@pytest.mark.timeout(900)
def test_c4_batch_pairs_vs_oracle(oracle):
    """C4 (BASELINE configs[3]): >= 4 distinct pairs of the bench's device-generated set registered by ONE
    ndt_align_batch call (several streams in flight), each compared with the oracle on the same points (copied back)."""
    import ctypes as C
    from xchu_slam_amd import synth
    wl = bench.WORKLOADS["c4"]
    idx = [0, 1, 2, 3, 4]
    g = xa.NormalDistributionsTransform()
    g.setResolution(1.0)
    g.setTransformationEpsilon(0.0)
    g.setMaximumIterations(3)
    lib = g._lib
    d_world = g.device_upload(np.zeros(65536, np.float32))
    pairs, hosts, specs = [], [], []
    for i in idx:
        spec = synth.c4_pair_spec(i, half=wl["half"], density=wl["density"], n_source=wl["n_source"], max_range=wl["max_range"])
        buf = g.device_upload(np.zeros((spec.n_target + spec.n_source, 4), np.float32))
        dt, ds = buf, buf + 16 * spec.n_target
        synth.generate_pair_device(spec, 0, d_world, dt, ds)
        t = np.empty((spec.n_target, 4), np.float32)
        s = np.empty((spec.n_source, 4), np.float32)
        lib.ndt_memcpy_d2h(g.ctx, t.ctypes.data_as(C.c_void_p), C.c_void_p(dt), t.nbytes)
        lib.ndt_memcpy_d2h(g.ctx, s.ctypes.data_as(C.c_void_p), C.c_void_p(ds), s.nbytes)
        assert np.all(np.isfinite(t)) and np.all(np.isfinite(s))
        pairs.append((dt, spec.n_target, ds, spec.n_source, spec.guess))
        hosts.append((t[:, :3].copy(), s[:, :3].copy()))
        specs.append(spec)
    res = g.align_batch(pairs)
    # the same pair generated twice is the same bits (pair i is a pure function of its seeds)
    spec0 = specs[0]
    buf = g.device_upload(np.zeros((spec0.n_target + spec0.n_source, 4), np.float32))
    synth.generate_pair_device(spec0, 0, d_world, buf, buf + 16 * spec0.n_target)
    s4 = np.empty((spec0.n_source, 4), np.float32)
    lib.ndt_memcpy_d2h(g.ctx, s4.ctypes.data_as(C.c_void_p), C.c_void_p(buf + 16 * spec0.n_target), s4.nbytes)
    assert np.array_equal(s4[:, :3], hosts[0][1])
    for k, i in enumerate(idx):
        tgt, src = hosts[k]
        o = oracle.OracleNDT(num_threads=NT, resolution=1.0, step_size=0.1, trans_eps=0.0, max_iter=3)
        o.set_target(tgt)
        o.set_source(src)
        ro = o.align(specs[k].guess)
        nv = int(sum(1 for n in o.grid_leaves()["npts"] if n >= 6))
        o.close()
        r = res[k]
        assert 150_000 < nv < 260_000                      # ~200k valid voxels
        assert r["nr_iterations"] == ro["nr_iterations"] and r["converged"] == ro["converged"]
        assert np.max(np.abs(r["final_tf"] - ro["final_tf"])) < TF_TOL
        assert r["n_pairs"] == ro["n_pairs"]
        t_err, _ = pose_err(r["final_tf"], specs[k].true_pose)
        assert t_err < 0.5
    g.close()
