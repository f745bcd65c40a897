"""C3 parity at its own size (BASELINE configs[2]): the first 100 scans of the bench's C3 sequence —
120 000-point synthetic HDL-64-like scans at consecutive KITTI-00 ground-truth poses, the same world, seed and scan
generator as `bench.py --workload c3` — streamed through the native odom_node scan loop on the GPU
(include/ndt_odom.h: ndt_odom_process_device, and the bench's pipelined ndt_odom_process_batch_device, which must
give the same records field for field) and through the CPU restatement of the same loop over the oracle
(tests/odom_restate.py, all host threads).

Per scan: keyframe and localmap-reset decisions exact (odom_node.cpp:321-356), t_localizer within 1e-6 m / 1e-6 rad
(f32 transforms; only the f64 reduction orders differ; north star 1e-4), iteration counts and convergence flags equal.
"""
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

N_SCANS = 100
N_POINTS = 120_000


@pytest.fixture(scope="module")
def c3_scans():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    workers = max(1, min(16, (os.cpu_count() or 2) - 1))
    return bench.make_c3_scans(N_SCANS, N_POINTS, seed=0, workers=workers)


def _rot_err(A, B):
    d = A[:3, :3].astype(np.float64).T @ B[:3, :3].astype(np.float64)
    return float(np.linalg.norm([d[2, 1] - d[1, 2], d[0, 2] - d[2, 0], d[1, 0] - d[0, 1]]) / 2)


def test_c3_replay_100_scans_at_size(c3_scans, oracle):
    import odom_restate as R
    import xchu_slam_amd as xa
    odom = xa.LidarOdom(ndt_resolution=1.0)
    dev = [odom.upload(s) for s in c3_scans]
    g = [odom.process_device(ptr, n, 0.1 * k) for k, (ptr, n) in enumerate(dev)]
    odom.close()
    # the bench's pipelined replay (ndt_odom_process_batch_device): the same records, field for field
    odom = xa.LidarOdom(ndt_resolution=1.0)
    dev = [odom.upload(s) for s in c3_scans]
    gb = odom.process_batch_device(dev, [0.1 * k for k in range(len(dev))])
    odom.close()
    for k, (a, b) in enumerate(zip(g, gb)):
        for f in a:
            if not f.startswith("ms_"):
                assert np.array_equal(a[f], b[f]), (k, f, a[f], b[f])
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    o = R.OdomRestatement(ndt_resolution=1.0, num_threads=min(threads, os.cpu_count() or 1))
    c = [o.process(s) for s in c3_scans]
    o.close()
    assert len(g) == len(c) == N_SCANS
    assert sum(r["keyframe"] for r in c) >= 20 and sum(r["localmap_reset"] for r in c) >= 2
    worst_t = worst_r = 0.0
    for k, (a, b) in enumerate(zip(g, c)):
        assert a["keyframe"] == b["keyframe"], k
        assert a["localmap_reset"] == b["localmap_reset"], k
        dt = float(np.abs(a["t_localizer"][:3, 3] - b["t_localizer"][:3, 3]).max())
        dr = _rot_err(a["t_localizer"], b["t_localizer"])
        worst_t, worst_r = max(worst_t, dt), max(worst_r, dr)
        assert dt < 1e-6 and dr < 1e-6, (k, dt, dr)
        assert a["final_num_iteration"] == b["final_num_iteration"], (k, a["final_num_iteration"], b["final_num_iteration"])
        assert a["has_converged"] == b["has_converged"], k
    print(f"c3 100 x 120k: worst |dt| {worst_t:.2e} m, worst rot {worst_r:.2e} rad, "
          f"{sum(r['keyframe'] for r in c)} keyframes, {sum(r['localmap_reset'] for r in c)} localmap resets")
