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
