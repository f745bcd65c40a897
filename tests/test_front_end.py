"""filter_node front end (xchu_mapping/src/filter_node.cpp:218-273): NaN removal, range crop,
pcl::VoxelGrid(0.5), pcl::StatisticalOutlierRemoval(30, 1.0).

CPU: the oracle's grid k-NN against brute force (bit-identical distances), the crop + voxel stages against numpy, a
known-answer SOR case.  GPU (`-m gpu`): the device pipeline against the oracle — same kept points bit for bit, same
per-point SOR distances bit for bit (identical float squared distances, ascending double sum), threshold within
1e-12 (fixed-order vs sequential f64 sums).  Parity unpinned against PCL itself (not vendored, not runnable here)."""
import numpy as np
import pytest

from helpers import raw_scan


def test_oracle_grid_knn_matches_brute(oracle):
    cloud = raw_scan(seed=4, n_points=12000, n_outliers=60)
    og, dg, tg, nvg = oracle.filter_scan(cloud, brute=False, is_dense=False)
    ob, db, tb, nvb = oracle.filter_scan(cloud, brute=True, is_dense=False)
    assert nvg == nvb > 1000
    assert np.array_equal(dg, db)
    assert np.array_equal(og, ob)
    assert tg[0] == tb[0]


def test_oracle_crop_and_voxel_vs_numpy(oracle):
    cloud = raw_scan(seed=5, n_points=8000, n_outliers=40)
    fin = np.isfinite(cloud[:, :3]).all(1)
    c = cloud[fin]
    r = np.sqrt(c[:, 0].astype(np.float64) ** 2 + c[:, 1].astype(np.float64) ** 2)
    crop = c[(r > 1.0) & (r < 60.0)]
    ds = oracle.voxel_downsample(crop, 0.5)
    # SOR disabled by a huge multiplier: the output is the voxel-filtered cloud
    out, dist, thr, nv = oracle.filter_scan(cloud, stddev_mul=1e30, is_dense=False)
    assert nv == len(ds) and np.array_equal(out, ds)


def test_oracle_sor_known_answer(oracle):
    """A dense 20 m x 20 m plane sampled at 0.5 m plus 5 isolated points 10 m above it: the isolated points (mean
    neighbour distance ~10 m) are removed, every plane point is kept."""
    g = np.stack(np.meshgrid(np.arange(-10, 10, 0.5) + 0.25, np.arange(-10, 10, 0.5) + 0.25), -1).reshape(-1, 2)
    g = g[np.hypot(g[:, 0], g[:, 1]) > 1.5]
    plane = np.concatenate([g, np.zeros((len(g), 1))], 1)
    iso = np.array([[15, 15, 10], [-15, 15, 10], [15, -15, 10], [-15, -15, 10], [0, 20, 10]], np.float64) + 0.25
    pts = np.concatenate([plane, iso]).astype(np.float32)
    cloud = np.concatenate([pts, np.ones((len(pts), 1), np.float32)], 1)
    out, dist, thr, nv = oracle.filter_scan(cloud)
    assert nv == len(cloud)
    assert len(out) == len(plane)
    assert not np.isin(out[:, 2], [10.25]).any()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n", [(7, 30000), (8, 120000)])
def test_filter_scan_matches_oracle(oracle, seed, n):
    xa = pytest.importorskip("xchu_slam_amd")
    cloud = raw_scan(seed=seed, n_points=n, n_outliers=n // 200)
    od, odist, othr, onv = oracle.filter_scan(cloud, is_dense=False)
    gd, gdist, gthr, gnv = xa.filter_scan(cloud, stats=True)
    assert gnv == onv
    assert np.array_equal(gdist, odist)
    assert abs(gthr[0] - othr[0]) <= 1e-12 * abs(othr[0])
    assert len(gd) == len(od) and np.array_equal(gd, od)
    assert len(od) < onv  # outliers were removed


@pytest.mark.gpu
def test_filter_scan_edges(oracle):
    xa = pytest.importorskip("xchu_slam_amd")
    empty = np.zeros((0, 4), np.float32)
    assert xa.filter_scan(empty).shape == (0, 4)
    # everything cropped away
    near = np.array([[0.1, 0.2, 0.0, 1.0], [0.5, 0.5, 1.0, 1.0]], np.float32)
    assert xa.filter_scan(near).shape == (0, 4)
    # fewer voxels than mean_k: voxel output returned without outlier removal
    few = np.array([[5.0 + i, 3.0, 0.0, 0.5] for i in range(10)], np.float32)
    od, _, _, onv = oracle.filter_scan(few)
    gd = xa.filter_scan(few)
    assert onv == 10 and np.array_equal(gd, od)


def test_oracle_ror_known_answer(oracle):
    """RadiusOutlierRemoval(0.8, 5): a 0.5 m lattice plane keeps every point (>= 5 within 0.8 m counting itself: the
    4 edge neighbours at 0.5 m, the 4 diagonal at 0.71 m), an isolated pair floating above it is removed."""
    g = np.stack(np.meshgrid(np.arange(-10, 10, 0.5) + 0.25, np.arange(-10, 10, 0.5) + 0.25), -1).reshape(-1, 2)
    g = g[np.hypot(g[:, 0], g[:, 1]) > 1.5]
    plane = np.concatenate([g, np.zeros((len(g), 1))], 1)
    iso = np.array([[5.25, 5.25, 6.25], [5.25, 5.75, 6.25]])
    pts = np.concatenate([plane, iso]).astype(np.float32)
    cloud = np.concatenate([pts, np.ones((len(pts), 1), np.float32)], 1)
    out, _, _, nv = oracle.filter_scan(cloud, outlier_method=1)
    assert nv == len(cloud)
    # lattice corners have 3 neighbours + itself = 4 < 5 -> removed; all interior lattice points kept
    assert len(out) < len(plane) and not np.isin(out[:, 2], [6.25]).any()


@pytest.mark.gpu
def test_filter_scan_ror_matches_oracle(oracle):
    xa = pytest.importorskip("xchu_slam_amd")
    cloud = raw_scan(seed=9, n_points=20000, n_outliers=100)
    od, _, _, onv = oracle.filter_scan(cloud, is_dense=False, outlier_method=1)
    gd = xa.filter_scan(cloud, outlier_method=1)
    assert len(gd) == len(od) and np.array_equal(gd, od)
    assert len(od) < onv
