"""Generate the committed golden fixtures from the CPU oracle (1 thread => deterministic).

The reference has no golden vectors for this path, so these fixtures pin the restatement
itself (regression) and give the GPU a fixed, file-based target.  Inputs are the seeded synthetic clouds.
Run: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_lib  # noqa: E402
from helpers import small_pair  # noqa: E402

CASES = {
    "direct7_eps0": dict(resolution=1.0, step_size=0.1, trans_eps=0.0, max_iter=8, search=2),
    "direct7_eps001": dict(resolution=1.0, step_size=0.1, trans_eps=0.01, max_iter=30, search=2),
    "kdtree_res2": dict(resolution=2.0, step_size=0.1, trans_eps=0.01, max_iter=10, search=0),
    "pclndt_f64": dict(resolution=1.0, step_size=0.1, trans_eps=0.01, max_iter=10, search=0, precision_mode=1),
    "mt_inner_loop": dict(resolution=1.0, step_size=0.01, trans_eps=0.5, max_iter=3, search=2),
}


def main():
    pair = small_pair(seed=21, half=18.0, density=6.0, n_source=1500, max_range=15.0)
    out = {"target": pair.target, "source": pair.source, "guess": pair.guess.astype(np.float32),
           "true_pose": pair.true_pose}
    for name, prm in CASES.items():
        o = oracle_lib.OracleNDT(num_threads=1, **prm)
        o.set_target(pair.target)
        o.set_source(pair.source)
        r = o.align(pair.guess)
        h = o.history()
        out[f"{name}/final_tf"] = r["final_tf"]
        out[f"{name}/meta"] = np.array([r["nr_iterations"], r["converged"], r["n_passes"], r["n_pairs"]], np.int64)
        out[f"{name}/trans_probability"] = np.array(r["trans_probability"])
        out[f"{name}/hist_x"] = np.stack([x["x"] for x in h])
        out[f"{name}/hist_score"] = np.array([x["score"] for x in h])
        out[f"{name}/hist_g"] = np.stack([x["g"] for x in h])
        out[f"{name}/hist_H"] = np.stack([x["H"] for x in h])
        out[f"{name}/hist_kind"] = np.array([x["kind"] for x in h], np.int32)
        out[f"{name}/hist_pairs"] = np.array([x["pairs"] for x in h], np.int64)
        out[f"{name}/params"] = np.array([prm.get(k, d) for k, d in [("resolution", 1.0), ("step_size", 0.1), ("trans_eps", 0.1),
                                                                  ("max_iter", 35), ("search", 2), ("precision_mode", 0)]])
    o = oracle_lib.OracleNDT(num_threads=1)
    o.set_target(pair.target)
    lv = o.grid_leaves()
    for k in ("keys", "npts", "mean", "icov", "centroid"):
        out[f"grid/{k}"] = lv[k]
    out["grid/header"] = np.array([*o.grid_header()["min_b"], *o.grid_header()["max_b"], *o.grid_header()["div_b"]], np.int64)
    rng = np.random.default_rng(9)
    ds_in = np.concatenate([pair.target[:4000], rng.uniform(0, 255, (4000, 1)).astype(np.float32)], 1)
    out["downsample/input"] = ds_in
    out["downsample/leaf1"] = oracle_lib.voxel_downsample(ds_in, 1.0)
    np.savez_compressed(os.path.join(HERE, "ndt_small.npz"), **out)
    print("wrote", os.path.join(HERE, "ndt_small.npz"), sum(v.nbytes for v in out.values()), "bytes raw")


if __name__ == "__main__":
    main()
