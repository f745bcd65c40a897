"""Merge-extended targets (ndt_set_target_append_device, k_merge_append): odom_node's setInputTarget(pc_target_) between
localmap resets hands over the localmap, which only grows by appends (odom_node.cpp:233, 349).  The grid built by merging
the new points' sort into the current one must be the grid a fresh setInputTarget builds over the same points, bit for
bit (voxel_grid_covariance_omp_impl.hpp:67-367: the stable sort is what fixes each voxel's f64 summation order).
"""
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _grids_equal(a, b, what):
    ia, ib = a.grid_info(), b.grid_info()
    assert ia == ib, (what, ia, ib)
    la, lb = a.grid_leaves(), b.grid_leaves()
    for k in ("keys", "npts", "mean", "icov", "centroid"):
        assert np.array_equal(la[k], lb[k]), (what, k)
    return ia


def _world_points(seed=7, n_max=420_000):
    from xchu_slam_amd import synth
    w = synth.make_world(seed, half=120.0)
    p = synth.to_xyz4(w.target(6.0, seed + 1))
    return p[:n_max]


def test_append_grid_matches_fresh_build():
    """Chunks appended in x order grow the box at its high end; the last chunk also holds the lowest-x points, so the
    box grows at its low end too (every old key re-expressed); an empty append and a parameter change (which makes the
    next append a fresh build) are in the sequence."""
    import xchu_slam_amd as xa
    pts = _world_points()
    order = np.argsort(pts[:, 0], kind="stable")
    low = order[:3000]
    rest = order[3000:]
    rng = np.random.default_rng(3)
    cuts = [240_000, 270_000, 270_000, 281_000, len(rest)]
    chunks, start = [], 0
    for c in cuts:
        ch = rest[start:c].copy()
        rng.shuffle(ch)
        chunks.append(ch)
        start = c
    chunks[-1] = np.concatenate([chunks[-1], low])
    rng.shuffle(chunks[-1])
    seq = np.ascontiguousarray(pts[np.concatenate(chunks)])
    a = xa.NormalDistributionsTransform()
    b = xa.NormalDistributionsTransform()
    for g in (a, b):
        g.setResolution(1.0)
        g.setNeighborhoodSearchMethod(xa.DIRECT7)
    d = a.device_upload(seq)
    try:
        n = len(chunks[0])
        a.setInputTargetDevice(d, n)
        b.setInputTargetDevice(d, n)
        _grids_equal(a, b, "first")
        boxes = [a.grid_info()["div_b"]]
        mins = [a.grid_info()["min_b"]]
        for k, ch in enumerate(chunks[1:], 1):
            if k == 3:
                for g in (a, b):  # a parameter change: the next append is built from scratch
                    g.setMinPointPerVoxel(6)
            a.setInputTargetAppendDevice(d, n, len(ch))
            n += len(ch)
            b.setInputTargetDevice(d, n)
            info = _grids_equal(a, b, f"append {k}")
            boxes.append(info["div_b"])
            mins.append(info["min_b"])
        assert boxes[1] != boxes[0]        # grown at the high end (old keys re-expressed)
        assert mins[-1] != mins[-2]        # grown at the low end
        # the merge path actually ran (appends 1, 2 and 4; append 3 follows a parameter change: a full build), and the
        # fresh builds never merged (ndt_build_stats)
        sa, sb = a.build_stats(), b.build_stats()
        assert sa["merge"] == 3 and sa["full"] == 2 and sa["rerun"] == 0, sa
        assert sb["merge"] == 0 and sb["full"] == len(chunks), sb
        # the same grid registers the same way
        from xchu_slam_amd import synth
        w = synth.make_world(7, half=120.0)
        src = synth.to_xyz4(w.scan(60_000, (0.0, 0.0), 11, max_range=60.0))
        guess = np.eye(4, dtype=np.float32)
        guess[:3, 3] = (0.3, -0.2, 0.05)
        res = []
        for g in (a, b):
            g.setInputSource(src)
            g.align(guess, want_output=False)
            res.append(g.getFinalTransformation())
        assert np.array_equal(res[0], res[1])
    finally:
        a.device_free(d)
        a.close()
        b.close()


def test_append_after_other_sort_and_mismatch_falls_back():
    """A VoxelGrid filter on the same ctx reuses the main stream's sort scratch, and an n_old that is not the current
    target's size breaks the contract's precondition: both appends are built from scratch, still equal to fresh builds."""
    import xchu_slam_amd as xa
    pts = _world_points(seed=9, n_max=200_000)
    a = xa.NormalDistributionsTransform()
    b = xa.NormalDistributionsTransform()
    d = a.device_upload(pts)
    try:
        a.setInputTargetDevice(d, 150_000)
        xa.voxel_downsample(pts[:50_000], 0.5, ndt=a)
        a.setInputTargetAppendDevice(d, 150_000, 20_000)
        b.setInputTargetDevice(d, 170_000)
        _grids_equal(a, b, "after filter")
        a.setInputTargetAppendDevice(d, 160_000, 40_000)  # n_old != current size: fresh build over all 200k
        b.setInputTargetDevice(d, 200_000)
        _grids_equal(a, b, "mismatch")
    finally:
        a.device_free(d)
        a.close()
        b.close()


def test_append_new_points_stored_by_the_build():
    """d_new: the appended points are read from another buffer and stored after the old ones by the build (k_minmax),
    no separate copy; the grid equals a fresh build, and the target buffer holds the points afterwards."""
    import ctypes as C
    import xchu_slam_amd as xa
    pts = _world_points(seed=11, n_max=260_000)
    n0, n1 = 200_000, 60_000
    tgt = pts.copy()
    tgt[n0:] = 0.0  # the snapshot holds only the old points
    a = xa.NormalDistributionsTransform()
    b = xa.NormalDistributionsTransform()
    dt = a.device_upload(tgt)
    ds = a.device_upload(pts)
    try:
        a.setInputTargetDevice(dt, n0)
        a.setInputTargetAppendDevice(dt, n0, n1, d_new=ds + 16 * n0)
        b.setInputTargetDevice(ds, n0 + n1)
        _grids_equal(a, b, "d_new")
        back = np.zeros_like(pts)
        xa._lib.check(a._lib.ndt_memcpy_d2h(a.ctx, back.ctypes.data_as(C.c_void_p), C.c_void_p(dt), back.nbytes), a.ctx)
        assert np.array_equal(back, pts)
    finally:
        a.device_free(dt)
        a.device_free(ds)
        a.close()
        b.close()


@pytest.fixture(scope="module")
def c3_scans_short():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    workers = max(1, min(16, (os.cpu_count() or 2) - 1))
    return bench.make_c3_scans(60, 120_000, seed=0, workers=workers)


def test_odom_merge_matches_fresh_targets(c3_scans_short):
    """The odom_node loop with merge-extended keyframe targets (the default) against the same loop with every target
    built from scratch (NDT_NO_TARGET_MERGE): the records are identical field for field."""
    import ctypes as C
    import xchu_slam_amd as xa
    out, merges = [], []
    for env in (None, "1"):
        if env is None:
            os.environ.pop("NDT_NO_TARGET_MERGE", None)
        else:
            os.environ["NDT_NO_TARGET_MERGE"] = env
        try:
            odom = xa.LidarOdom(ndt_resolution=1.0)
            dev = [odom.upload(s) for s in c3_scans_short]
            out.append(odom.process_batch_device(dev, [0.1 * k for k in range(len(dev))]))
            st = (C.c_longlong * 6)()
            xa._lib.check(odom._lib.ndt_build_stats(odom._ctx, st))
            merges.append(st[1])
            odom.close()
        finally:
            os.environ.pop("NDT_NO_TARGET_MERGE", None)
    g, f = out
    assert sum(r["keyframe"] for r in g) >= 20 and sum(r["localmap_reset"] for r in g) >= 1
    # the default loop extended its targets by merge, the NDT_NO_TARGET_MERGE loop never did
    assert merges[0] >= 10 and merges[1] == 0, merges
    for k, (a, b) in enumerate(zip(g, f)):
        for fld in a:
            if not fld.startswith("ms_"):
                assert np.array_equal(a[fld], b[fld]), (k, fld, a[fld], b[fld])


def test_odom_late_fitness_query_matches(c3_scans_short):
    """getFitnessScore queued after the next target's build (NDT_ODOM_FIT_LATE: ndt_fitness_score_async_aligned against
    the aligned target's index) gives the records of the query queued before setInputTarget (odom_node.cpp:280, 349)."""
    import xchu_slam_amd as xa
    out = []
    for env in (None, "1"):
        if env is None:
            os.environ.pop("NDT_ODOM_FIT_LATE", None)
        else:
            os.environ["NDT_ODOM_FIT_LATE"] = env
        try:
            odom = xa.LidarOdom(ndt_resolution=1.0)
            dev = [odom.upload(s) for s in c3_scans_short]
            out.append(odom.process_batch_device(dev, [0.1 * k for k in range(len(dev))]))
            odom.close()
        finally:
            os.environ.pop("NDT_ODOM_FIT_LATE", None)
    g, f = out
    assert any(r["keyframe"] for r in g)
    for k, (a, b) in enumerate(zip(g, f)):
        for fld in a:
            if not fld.startswith("ms_"):
                assert np.array_equal(a[fld], b[fld]), (k, fld, a[fld], b[fld])
