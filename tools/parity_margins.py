"""Parity margins on the GPU: how far the HIP path is from the oracle where the tests only assert a bar.  For each case,
the max per-pass |x_dev - x_oracle| over a whole align, the final transform difference, the largest pair-count
difference, and one pass at the guess (score / g / H relative error).  The oracle evaluates exp / sin / cos as the
shipped libndt_omp.so's model (exp_mode 1, trig_mode 1: (float)exp((double)x), sin / cos rounded once).  Writes one JSON object (stdout, and argv[1] when given).
   python tools/parity_margins.py gpurun_out/parity_margins.json"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import xchu_slam_amd as xa  # noqa: E402
import oracle_lib  # noqa: E402
from helpers import rel_err, small_pair  # noqa: E402
import bench  # noqa: E402


def case(name, target, source, guess, threads, **prm):
    o = oracle_lib.OracleNDT(num_threads=threads, **prm)
    o.set_target(target)
    o.set_source(source)
    g = xa.NormalDistributionsTransform()
    for k, v in prm.items():
        setattr(g._params, k, v)
    g._push()
    g.setInputTarget(target)
    g.setInputSource(source)
    p = oracle_lib.initial_p(guess)
    T = guess.astype(np.float32)
    so, go, Ho, Po = o.derivatives(p, T, True)
    sg, gg, Hg, Pg = g.computeDerivatives(p, T, True)
    ro = o.align(guess)
    g.align(guess, want_output=False)
    rg = g.result()
    ho, hg = o.history(), g.history()
    same_passes = len(ho) == len(hg) and all(a["kind"] == b["kind"] for a, b in zip(ho, hg))
    dx = [float(np.max(np.abs(np.asarray(a["x"]) - np.asarray(b["x"])))) for a, b in zip(ho, hg)]
    dp = [abs(int(a["pairs"]) - int(b["pairs"])) for a, b in zip(ho, hg)]
    return name, {
        "passes": len(ho), "same_pass_sequence": bool(same_passes),
        "iterations": [int(ro["nr_iterations"]), int(rg["nr_iterations"])],
        "max_pass_dx": max(dx) if dx else None, "pass_dx_exact_zero": int(sum(1 for d in dx if d == 0.0)),
        "max_pair_count_diff": max(dp) if dp else None,
        "final_tf_maxdiff": float(np.max(np.abs(rg["final_tf"] - ro["final_tf"]))),
        "single_pass": {"P_equal": bool(Po == Pg), "score_rel": abs(so - sg) / abs(so), "g_rel": rel_err(gg, go),
                        "H_rel": rel_err(Hg, Ho)},
    }


def main():
    oracle_lib.build_oracle()
    out = {}
    pair = small_pair()
    for nm, search in (("small_direct7", xa.DIRECT7), ("small_direct26", xa.DIRECT26), ("small_direct1", xa.DIRECT1),
                       ("small_kdtree", xa.KDTREE)):
        k, v = case(nm, pair.target, pair.source, pair.guess, 1, resolution=1.0, step_size=0.1, trans_eps=0.0, max_iter=30,
                    search=search)
        out[k] = v
        print(k, v, flush=True)
    c2 = bench.make_pool(0, 1, bench.WORKLOADS["c2"])[0]
    k, v = case("c2_full_size", c2.target, c2.source, c2.guess, 16, resolution=1.0, step_size=0.1, trans_eps=0.0,
                max_iter=30, search=xa.DIRECT7)
    out[k] = v
    print(k, v, flush=True)
    line = json.dumps(out)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(line + "\n")
    print(line)


if __name__ == "__main__":
    main()
