"""Distribution of getFitnessScore's nearest-neighbour distances in the C3 loop (how many queries leave k_fitness's
3x3x3 / 5x5x5 cell cubes for the block-shell search): odom over the first scans of the C3 sequence, then the last
scan against the target it was aligned to.   python tools/fit_dist_probe.py [n_scans]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
import xchu_slam_amd as xa  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    scans = bench.make_c3_scans(n, 120_000, seed=0, workers=8)
    odom = xa.LidarOdom(ndt_resolution=1.0)
    recs = [odom.process(s, 0.1 * k) for k, s in enumerate(scans[:-1])]
    tgt = odom.cloud(2)  # the registration's current target (pc_target_)
    odom.close()
    r = xa.NormalDistributionsTransform()
    r.setResolution(1.0)
    r.setInputTarget(tgt)
    r.setInputSource(scans[-1])
    r.align(recs[-1]["t_localizer"], want_output=False)
    score, d2 = r.getFitnessScore(return_distances=True)
    d = np.sqrt(d2.astype(np.float64))
    print(f"target {len(tgt)} pts, query {len(d)} pts, score {score:.4f}")
    for q in (50, 75, 90, 95, 99, 99.9):
        print(f"  p{q}: {np.percentile(d, q):.3f} m")
    for t in (1.0, 2.0, 3.0, 8.0, 16.0):
        print(f"  > {t:4.1f} m: {np.mean(d > t) * 100:.2f} %")
    r.close()


if __name__ == "__main__":
    main()
