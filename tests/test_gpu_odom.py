"""GPU parity of the native odom_node replay driver (include/ndt_odom.h, csrc/odom_estimate.cpp) against the CPU
restatement of the same scan loop over the oracle registration (tests/odom_restate.py).

Sequence: synthetic scans of a seeded world taken at consecutive KITTI-00 ground-truth poses (SURVEY §8d C3;
tests/golden/kitti00_gt.npz), odom_node defaults except ndt_resolution 1.0.
Tolerances: registration parity is 1e-6 m / 1e-6 rad per scan (f32 transforms; only the f64 reduction order differs
between device and oracle, measured ~1e-15 in the per-pass parameters); the Pose6D helpers (Pose6D2Matrix,
Matrix2Pose6D) and the keyframe/localmap bookkeeping are exact.
"""
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

N_SCANS = 16
N_POINTS = 20000


@pytest.fixture(scope="module")
def sequence():
    from xchu_slam_amd import synth
    tum = np.load(os.path.join(ROOT, "tests", "golden", "kitti00_gt.npz"))["tum"]
    return synth.make_sequence(tum, N_SCANS, N_POINTS, seed=11, start=120)


@pytest.fixture(scope="module")
def gpu_run(sequence):
    import xchu_slam_amd as xa
    _, poses, scans = sequence
    odom = xa.LidarOdom(ndt_resolution=1.0)
    recs = [odom.process(s, 0.1 * k) for k, s in enumerate(scans)]
    clouds = {w: odom.cloud(w) for w in (0, 1, 2)}
    odom.close()
    return recs, clouds


@pytest.fixture(scope="module")
def cpu_run(sequence, oracle):
    import odom_restate as R
    _, poses, scans = sequence
    o = R.OdomRestatement(ndt_resolution=1.0)
    recs = [o.process(s) for s in scans]
    clouds = {0: o.localmap, 1: o.tmp_map}
    o.close()
    return recs, clouds


def _rot_err(A, B):
    # small-angle rotation difference (rad) from the skew part of A^T B
    d = A[:3, :3].astype(np.float64).T @ B[:3, :3].astype(np.float64)
    return float(np.linalg.norm([d[2, 1] - d[1, 2], d[0, 2] - d[2, 0], d[1, 0] - d[0, 1]]) / 2)


def test_replay_matches_restatement(gpu_run, cpu_run):
    g, _ = gpu_run
    c, _ = cpu_run
    assert len(g) == len(c) == N_SCANS
    for k, (a, b) in enumerate(zip(g, c)):
        assert a["keyframe"] == b["keyframe"], k
        assert a["localmap_reset"] == b["localmap_reset"], k
        assert np.abs(a["t_localizer"][:3, 3] - b["t_localizer"][:3, 3]).max() < 1e-6, (k, a["t_localizer"], b["t_localizer"])
        assert _rot_err(a["t_localizer"], b["t_localizer"]) < 1e-6, k
        assert np.allclose(a["current_pose"], b["current_pose"], atol=1e-6), k
        assert a["final_num_iteration"] == b["final_num_iteration"], k
        assert a["has_converged"] == b["has_converged"], k
        assert a["n_appended"] == b["n_appended"], k


def test_pose_helpers_exact(gpu_run):
    """Pose6D2Matrix / Matrix2Pose6D / t_base_link in the C++ driver = the restatement, bit for bit."""
    import odom_restate as R
    g, _ = gpu_run
    for k, a in enumerate(g):
        assert np.array_equal(R.pose_to_matrix(a["guess_pose"]), a["init_guess"]), k
        assert np.array_equal(R.mul4(a["t_localizer"], np.eye(4, dtype=np.float32)), a["t_base_link"]), k
        assert np.array_equal(R.matrix_to_pose(a["t_base_link"]), a["current_pose"]), k
        assert np.array_equal(R.matrix_to_pose(a["t_localizer"]), a["localizer_pose"]), k
    # constant-velocity guess (odom_node.cpp:234-236): previous + diff, roll/pitch held
    for k in range(2, len(g)):
        prev, diff = g[k - 1]["current_pose"], g[k - 1]["diff_pose"]
        exp = prev + diff
        exp[3], exp[4] = prev[3], prev[4]
        assert np.array_equal(exp, g[k]["guess_pose"]), k


def test_bookkeeping_and_clouds(gpu_run, cpu_run):
    g, gc = gpu_run
    c, cc = cpu_run
    for k, (a, b) in enumerate(zip(g, c)):
        assert abs(a["n_localmap"] - b["n_localmap"]) <= max(4, b["n_localmap"] // 500), k
        assert abs(a["n_tmp_map"] - b["n_tmp_map"]) <= max(4, b["n_tmp_map"] // 500), k
        assert 0.0 < a["fitness_score"] < 1.0, k
    assert len(gc[0]) == g[-1]["n_localmap"] and len(gc[1]) == g[-1]["n_tmp_map"]
    assert len(gc[2]) == g[-1]["n_target"]
    # first scan seeds localmap with the full scan (odom_node.cpp:218-231)
    assert g[0]["n_localmap"] == N_POINTS and not g[0]["keyframe"]
    if len(gc[0]) == len(cc[0]):
        assert np.abs(gc[0][:, :3] - cc[0][:, :3]).max() < 1e-3


def test_replay_tracks_ground_truth(gpu_run, sequence):
    _, poses, _ = sequence
    g, _ = gpu_run
    P0 = np.linalg.inv(poses[0])
    for k, a in enumerate(g):
        gt = P0 @ poses[k]
        assert np.linalg.norm(a["t_localizer"][:3, 3] - gt[:3, 3]) < 0.15, k


def test_device_input_matches_host_input(sequence, gpu_run):
    import xchu_slam_amd as xa
    _, _, scans = sequence
    g, _ = gpu_run
    odom = xa.LidarOdom(ndt_resolution=1.0)
    for k, s in enumerate(scans[:6]):
        ptr, n = odom.upload(s)
        r = odom.process_device(ptr, n, 0.1 * k)
        assert np.array_equal(r["t_localizer"], g[k]["t_localizer"]), k
        assert r["n_localmap"] == g[k]["n_localmap"] and r["fitness_score"] == g[k]["fitness_score"], k
    odom.close()


def test_empty_scan_rejected():
    import xchu_slam_amd as xa
    from xchu_slam_amd import _lib
    odom = xa.LidarOdom()
    with pytest.raises(_lib.NdtError):
        odom.process(np.zeros((0, 3), np.float32), 0.0)
    odom.close()


def test_keyframe_insert_matches_voxel_downsample(sequence):
    """ndt_keyframe_insert_async = transformPointCloud + VoxelGrid + two appends (odom_node.cpp:290, 333-338):
    bit-identical to the synchronous VoxelGrid of the same transformed scan, appended behind existing points."""
    import ctypes as C

    import odom_restate as R
    import oracle_lib
    import xchu_slam_amd as xa
    _, _, scans = sequence
    g = xa.NormalDistributionsTransform()
    lib, ctx = g._lib, g._ctx
    scan = np.zeros((len(scans[3]), 4), np.float32)
    scan[:, :3] = scans[3]
    scan[:, 3] = np.arange(len(scan)) % 97  # intensity carried through the mean
    T = np.array([[0.8, -0.6, 0.0, 12.5], [0.6, 0.8, 0.0, -3.25], [0.0, 0.0, 1.0, 0.5], [0, 0, 0, 1]], np.float32)
    d_scan = g.device_upload(scan)
    pre_a, pre_b = 1000, 17
    d_a = g.device_upload(np.full((pre_a + len(scan), 4), 7.0, np.float32))
    d_b = g.device_upload(np.full((pre_b + len(scan), 4), 9.0, np.float32))
    Tc = np.ascontiguousarray(T.T).reshape(-1)
    st = lib.ndt_keyframe_insert_async(ctx, Tc.ctypes.data_as(C.POINTER(C.c_float)), d_scan, len(scan), 1.0, d_a, pre_a, d_b, pre_b)
    assert st == 0
    n = C.c_size_t()
    assert lib.ndt_keyframe_insert_result(ctx, C.byref(n)) == 0
    out_a = np.empty((pre_a + len(scan), 4), np.float32)
    out_b = np.empty((pre_b + len(scan), 4), np.float32)
    lib.ndt_memcpy_d2h(ctx, out_a.ctypes.data_as(C.c_void_p), d_a, out_a.nbytes)
    lib.ndt_memcpy_d2h(ctx, out_b.ctypes.data_as(C.c_void_p), d_b, out_b.nbytes)
    tr = R.transform_cloud(scan, T)
    ref = xa.voxel_downsample(tr, 1.0)
    assert n.value == len(ref)
    assert np.array_equal(out_a[pre_a:pre_a + n.value], ref) and np.array_equal(out_b[pre_b:pre_b + n.value], ref)
    assert np.all(out_a[:pre_a] == 7.0) and np.all(out_a[pre_a + n.value:] == 7.0) and np.all(out_b[:pre_b] == 9.0)
    # the oracle's VoxelGrid of the same points agrees to float rounding of the in-voxel sums
    orc = oracle_lib.voxel_downsample(tr, 1.0)
    assert len(orc) == n.value and np.allclose(orc, ref, atol=1e-4)
    for p in (d_scan, d_a, d_b):
        g.device_free(p)
    g.close()


def test_fitness_async_matches_sync(sequence):
    import xchu_slam_amd as xa
    _, _, scans = sequence
    g = xa.NormalDistributionsTransform()
    g.setResolution(1.0)
    g.setInputTarget(np.concatenate([scans[0], scans[1]]))
    g.setInputSource(scans[2])
    import ctypes as C
    f_sync = g.getFitnessScore(T=np.eye(4, dtype=np.float32))
    T = np.ascontiguousarray(np.eye(4, dtype=np.float32)).reshape(-1)
    assert g._lib.ndt_fitness_score_async(g._ctx, T.ctypes.data_as(C.POINTER(C.c_float)), 1e300) == 0
    out = C.c_double()
    assert g._lib.ndt_fitness_score_result(g._ctx, C.byref(out)) == 0
    assert out.value == f_sync
    g.close()


@pytest.mark.parametrize("method,incremental", [(1, False), (1, True), (0, False)])
def test_replay_backends(oracle, method, incremental):
    """odom_node's other registration backends through the same native scan loop: ndt_method_type 1 (ndt_cpu, the
    launch default; with and without incremental_voxel_update = updateVoxelGrid at keyframes, odom_node.cpp:343-347)
    and 0 (pcl_ndt) — poses per scan vs the restatement over the oracle's backend, 1e-6 m / 1e-6 rad."""
    import odom_restate as R
    import xchu_slam_amd as xa
    from xchu_slam_amd import synth
    tum = np.load(os.path.join(ROOT, "tests", "golden", "kitti00_gt.npz"))["tum"]
    _, poses, scans = synth.make_sequence(tum, 8, N_POINTS, seed=13, start=800)   # ~0.9 m per scan: keyframes
    odom = xa.LidarOdom(ndt_resolution=1.0, method_type=method, incremental_voxel_update=int(incremental))
    g = [odom.process(s, 0.1 * k) for k, s in enumerate(scans)]
    odom.close()
    o = R.OdomRestatement(ndt_resolution=1.0, method_type=method, incremental_voxel_update=incremental)
    c = [o.process(s) for s in scans]
    o.close()
    assert sum(r["keyframe"] for r in c) >= 3
    for k, (a, b) in enumerate(zip(g, c)):
        assert a["keyframe"] == b["keyframe"], k
        assert np.abs(a["t_localizer"][:3, 3] - b["t_localizer"][:3, 3]).max() < 1e-6, k
        assert _rot_err(a["t_localizer"], b["t_localizer"]) < 1e-6, k
        assert a["final_num_iteration"] == b["final_num_iteration"], k


def test_replay_fitness_vs_kdtree(sequence):
    """getFitnessScore per scan (odom_node.cpp:280) inside the native loop, where its index is built on the fitness side
    stream beside the voxel build and the query runs beside the keyframe insertion and the next target build: each
    scan's score = the mean squared nearest-neighbour distance of the aligned scan to the target that scan was
    registered against (scipy cKDTree over that target, read back before the scan)."""
    from scipy.spatial import cKDTree

    import odom_restate as R
    import xchu_slam_amd as xa
    _, _, scans = sequence
    odom = xa.LidarOdom(ndt_resolution=1.0)
    target = None
    for k, s in enumerate(scans[:10]):
        r = odom.process(s, 0.1 * k)
        if k == 0:
            target = odom.cloud(2)  # the first scan seeds the target inside process()
        tr = R.transform_cloud(np.c_[s, np.zeros(len(s), np.float32)], r["t_localizer"])[:, :3].astype(np.float64)
        d, _ = cKDTree(target[:, :3].astype(np.float64)).query(tr)
        ref = float(np.mean(d * d))
        assert abs(r["fitness_score"] - ref) <= 1e-5 * ref, (k, r["fitness_score"], ref)
        target = odom.cloud(2)  # the next scan's target (set at this scan's keyframe)
    odom.close()


@pytest.mark.parametrize("method,incremental", [(3, False), (1, True)])
def test_batch_replay_matches_per_scan(sequence, method, incremental):
    """ndt_odom_process_batch_device (a scan's getFitnessScore and keyframe insertion collected after the next scan's
    align) = the per-scan calls, record for record (poses, fitness, keyframe/reset flags, cloud sizes); with ndt_cpu's
    incremental update nothing pends past a keyframe (updateVoxelGrid changes the next align's target)."""
    import xchu_slam_amd as xa
    _, _, scans = sequence
    recs = []
    for batch in (False, True):
        odom = xa.LidarOdom(ndt_resolution=1.0, method_type=method, incremental_voxel_update=int(incremental))
        dev = [odom.upload(s) for s in scans]
        if batch:
            recs.append(odom.process_batch_device(dev[:5], [0.1 * k for k in range(5)]) +
                        odom.process_batch_device(dev[5:], [0.1 * k for k in range(5, len(dev))]))
        else:
            recs.append([odom.process_device(p, n, 0.1 * k) for k, (p, n) in enumerate(dev)])
        clouds = [odom.cloud(w) for w in (0, 1, 2)]
        recs[-1].append({"clouds": clouds})
        odom.close()
    a, b = recs
    assert sum(r["keyframe"] for r in a[:-1]) >= 3
    for k, (x, y) in enumerate(zip(a[:-1], b[:-1])):
        for f in x:
            if not f.startswith("ms_"):
                assert np.array_equal(x[f], y[f]), (k, f, x[f], y[f])
    for ca, cb in zip(a[-1]["clouds"], b[-1]["clouds"]):
        assert np.array_equal(ca, cb)


def test_batch_failure_mid_sequence_settles(sequence):
    """a batch that fails at scan k (here: a scan size the C-ABI rejects) leaves nothing pending —
    the records before it are complete (getFitnessScore and the keyframe insertion of scan k-1 collected, its appended
    points counted), no pointer into the caller's freed record array survives, and the next calls carry on exactly as
    an uninterrupted per-scan replay does."""
    import ctypes as C

    import xchu_slam_amd as xa
    from xchu_slam_amd import _lib
    _, _, scans = sequence
    n_all, k = 16, 14  # the batch holds scans 0..13, scan 13 is rejected; scans 13..15 follow one by one
    ref = xa.LidarOdom(ndt_resolution=1.0)
    dev = [ref.upload(s) for s in scans[:n_all]]
    want = [ref.process_device(p, n, 0.1 * i) for i, (p, n) in enumerate(dev)]
    ref.close()

    odom = xa.LidarOdom(ndt_resolution=1.0)
    dev = [odom.upload(s) for s in scans[:n_all]]
    lib = _lib.load()
    ptrs = (C.c_void_p * k)(*[p for p, _ in dev[:k]])
    ns = (C.c_size_t * k)(*([n for _, n in dev[:k - 1]] + [1 << 31]))  # scan k-1: rejected by ndt_set_source_device
    st = (C.c_double * k)(*[0.1 * i for i in range(k)])
    out = (_lib.OdomResult * k)()
    assert lib.ndt_odom_process_batch_device(odom._h, ptrs, ns, st, k, out) == _lib.NDT_EINVAL
    got = [odom._record(out[i]) for i in range(k - 1)]
    del out, ptrs, ns, st  # the caller's record array is gone; nothing may still point into it
    for i in range(k - 1, n_all):
        got.append(odom.process_device(dev[i][0], dev[i][1], 0.1 * i))
    odom.close()
    assert any(r["keyframe"] for r in want[:k - 1])
    for i, (x, y) in enumerate(zip(got, want)):
        for f in x:
            if not f.startswith("ms_"):
                assert np.array_equal(x[f], y[f]), (i, f, x[f], y[f])
