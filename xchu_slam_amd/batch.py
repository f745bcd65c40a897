"""Batched offline replay: independent scan->localmap pairs sharded over ranks.

One process per GPU.  Pairs are independent units, so the only collective is one gather of the per-pair
result records at the end (RCCL over xGMI when the process group is "nccl", gloo on CPU).  The shard of
rank r is the contiguous block [r*P/W, (r+1)*P/W); each pair is registered by exactly the same device code
whatever the shard count, so results are bit-identical per pair for any W.
"""
from __future__ import annotations

from typing import Callable, Sequence

import numpy as np

RECORD_WIDTH = 16 + 4  # final_tf (row-major 4x4) + nr_iterations, converged, trans_probability, n_pairs


def shard_range(n_items: int, world: int, rank: int) -> range:
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    return range(rank * n_items // world, (rank + 1) * n_items // world)


def result_record(res: dict) -> np.ndarray:
    r = np.zeros(RECORD_WIDTH, np.float64)
    r[:16] = np.asarray(res["final_tf"], np.float64).reshape(-1)
    r[16] = res["nr_iterations"]
    r[17] = res["converged"]
    r[18] = res["trans_probability"]
    r[19] = res.get("n_pairs", 0)
    return r


def gather_records(local: np.ndarray, n_items: int, dist=None, device=None) -> np.ndarray:
    """All-gather each rank's (k_r, RECORD_WIDTH) block into the full (n_items, RECORD_WIDTH) table, in pair order."""
    if dist is None or not dist.is_initialized():
        return local
    import torch

    world = dist.get_world_size()
    kmax = max(len(shard_range(n_items, world, r)) for r in range(world))
    buf = np.zeros((kmax, RECORD_WIDTH), np.float64)
    buf[: len(local)] = local
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    out = np.zeros((n_items, RECORD_WIDTH), np.float64)
    for r in range(world):
        rg = shard_range(n_items, world, r)
        out[rg.start:rg.stop] = parts[r].cpu().numpy()[: len(rg)]
    return out


def replay(pairs: Sequence, align_fn: Callable[[object], dict], dist=None, device=None) -> np.ndarray:
    """Register this rank's shard of `pairs` with align_fn(pair) -> result dict, then gather every record."""
    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    mine = shard_range(len(pairs), world, rank)
    local = np.stack([result_record(align_fn(pairs[i])) for i in mine]) if len(mine) else np.zeros((0, RECORD_WIDTH))
    return gather_records(local, len(pairs), dist, device)


def gpu_align_fn(ndt) -> Callable[[object], dict]:
    """align_fn for synth.Pair objects on a NormalDistributionsTransform (one ctx per rank / device)."""

    def fn(pair):
        ndt.setInputTarget(pair.target)
        ndt.setInputSource(pair.source)
        ndt.align(pair.guess, want_output=False)
        return ndt.result()

    return fn
