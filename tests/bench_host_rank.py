"""bench.py's own launcher and C4 rank code (sharding, timing, one gather of the result records) driven with a HOST
aligner: the CPU oracle (test infrastructure) on small synthetic pairs.  Started by tests/test_distributed.py through
bench.spawn_ranks (gloo, world size 2) and as a single process; the GPU path of the same rank code is bench.GpuC4Backend."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import bench  # noqa: E402


class HostC4Backend:
    def __init__(self, dd, wl):
        self.pairs = {}

    def prepare(self, indices):
        from helpers import small_pair
        for i in indices:
            self.pairs[i] = small_pair(seed=100 + i, half=20.0, n_source=800)

    def run(self, indices):
        import oracle_lib
        out = []
        for i in indices:
            p = self.pairs[i]
            o = oracle_lib.OracleNDT(num_threads=1, trans_eps=0.0, max_iter=5)
            o.set_target(p.target)
            o.set_source(p.source)
            out.append(o.align(p.guess))
            o.close()
        return out

    def synchronize(self):
        pass

    def true_pose(self, i):
        return self.pairs[i].true_pose

    def describe(self):
        return {"aligner": "host oracle (test)"}


if __name__ == "__main__":
    sys.exit(bench.main(c4_backend=HostC4Backend))
