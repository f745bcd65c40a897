"""Multi-process (gloo, world size 2) checks of the batched replay path: contiguous sharding, one
gather of result records, results identical per pair for any shard count.  The per-pair aligner here is the
CPU oracle (test infrastructure); on the GPU box the same code runs with the HIP aligner (bench.py)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from xchu_slam_amd import batch


def test_shard_ranges_cover_exactly():
    for n in (0, 1, 7, 4096):
        for w in (1, 2, 3, 8):
            seen = []
            for r in range(w):
                seen.extend(batch.shard_range(n, w, r))
            assert seen == list(range(n))
    with pytest.raises(ValueError):
        batch.shard_range(10, 2, 2)


def _pairs():
    from helpers import small_pair
    return [small_pair(seed=s, half=20.0, n_source=800) for s in range(5)]


def _oracle_align(pair):
    import oracle_lib
    o = oracle_lib.OracleNDT(num_threads=1, trans_eps=0.0, max_iter=5)
    o.set_target(pair.target)
    o.set_source(pair.source)
    return o.align(pair.guess)


def _worker(rank, world, port, q):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    recs = batch.replay(_pairs(), _oracle_align, dist)
    q.put((rank, recs))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_world2_matches_single_process():
    single = batch.replay(_pairs(), _oracle_align, None)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0].shape == (5, batch.RECORD_WIDTH)
    assert np.array_equal(got[0], got[1])          # every rank holds the full table after the gather
    assert np.array_equal(got[0], single)          # bit-identical per pair for shard count 1 vs 2


def _run_bench_host(tmp_path, gpus):
    """bench.py --workload c4 through its own launcher (gpus > 1: bench.spawn_ranks) with the host aligner."""
    import json
    import subprocess
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench_host_rank.py")
    rec = str(tmp_path / f"rec{gpus}.npy")
    out = tmp_path / f"out{gpus}.txt"
    argv = ["--gpus", str(gpus), "--workload", "c4", "--steps", "5", "--warmup", "1", "--no-cpu-baseline", "--records-out", rec]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    with open(out, "w") as f:
        if gpus > 1:
            old = dict(os.environ)
            os.environ.clear()
            os.environ.update(env)
            try:
                rc = bench.spawn_ranks(gpus, argv, script=script, stdout=f)
            finally:
                os.environ.clear()
                os.environ.update(old)
        else:
            rc = subprocess.run([sys.executable, script, *argv], env=env, stdout=f, timeout=300).returncode
    assert rc == 0
    line = json.loads(out.read_text().strip().splitlines()[-1])
    return line, np.load(rec)


def test_bench_launcher_world2_matches_world1(tmp_path):
    one, rec1 = _run_bench_host(tmp_path, 1)
    two, rec2 = _run_bench_host(tmp_path, 2)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["scaling"] == "strong" and two["config"]["pairs_per_rank"] == [2, 3]
    assert rec1.shape == (5, batch.RECORD_WIDTH) and rec2.shape == rec1.shape
    assert np.array_equal(rec1, rec2)  # bit-identical per pair whatever the shard count
