"""The leading-tail pass chain (k_pass_lead: pass k's Newton step at the start of pass k+1's kernel, in every
workgroup) against the last-workgroup tails (k_pass_direct, ndt_set_pass_options(lead_tail=0)): the same pass records,
score, gradient, Hessian, iteration count and transform, bit for bit — both chains run the same arithmetic in the same
order, only where it runs differs.  Also covered: a multi-round align (the state and partials parities carried across
chain launches: an easy align first, so that the next one needs continuation rounds) and a DIRECT26 / DIRECT1 chain."""
import numpy as np
import pytest

from helpers import small_pair

pytestmark = pytest.mark.gpu

xa = pytest.importorskip("xchu_slam_amd")

CASES = [
    dict(name="direct7", seed=3, eps=0.0, iters=12, search=xa.DIRECT7, repeat=1),
    dict(name="direct7_repeat", seed=5, eps=0.01, iters=30, search=xa.DIRECT7, repeat=3),  # chain slots from the last align
    dict(name="direct26", seed=7, eps=0.0, iters=6, search=xa.DIRECT26, repeat=1),
    dict(name="direct1", seed=9, eps=0.0, iters=6, search=xa.DIRECT1, repeat=1),
    dict(name="continuation_rounds", seed=11, eps=0.001, iters=30, search=xa.DIRECT7, repeat=2, true_first=True),
]


def run_cases(lead_tail: bool):
    out = {}
    for case in CASES:
        pair = small_pair(seed=case["seed"])
        g = xa.NormalDistributionsTransform()
        g.set_pass_options(lead_tail=lead_tail)
        g.setResolution(1.0)
        g.setTransformationEpsilon(case["eps"])
        g.setMaximumIterations(case["iters"])
        g.setNeighborhoodSearchMethod(case["search"])
        g.setInputTarget(pair.target)
        g.setInputSource(pair.source)
        for k in range(case["repeat"]):
            # "true_first": an easy align first (guess = true pose, few passes), so that the next align's first chain
            # round is too short and continuation rounds (other ping-pong parity) follow
            g.align(pair.true_pose if (case.get("true_first") and k == 0) else pair.guess, want_output=False)
        r = g.result()
        out[case["name"]] = {"tf": r["final_tf"].astype(np.float64).ravel().tolist(), "iters": r["nr_iterations"],
                             "passes": r["n_passes"],
                             "hist": [[h["kind"], h["score"], h["pairs"]] + h["x"].tolist() + h["g"].tolist()
                                      + h["H"].ravel().tolist() for h in g.history()]}
        g.close()
    return out


@pytest.mark.timeout(300)
def test_lead_chain_matches_last_workgroup_tails():
    here, other = run_cases(True), run_cases(False)
    for case in CASES:
        a, b = here[case["name"]], other[case["name"]]
        assert a["iters"] == b["iters"] and a["passes"] == b["passes"], case["name"]
        if case.get("true_first"):
            assert a["passes"] > 8  # more passes than the first chain round after the easy align covers
        assert a["tf"] == b["tf"], case["name"]
        assert len(a["hist"]) == len(b["hist"]) > 0
        for ra, rb in zip(a["hist"], b["hist"]):
            assert ra == rb, case["name"]
