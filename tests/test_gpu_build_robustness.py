"""Robustness of the target build and of the align-graph cache (no reference counterpart: the reference's
VoxelGridCovariance::applyFilter, voxel_grid_covariance_omp_impl.hpp:208-264, is a serial std::map insert; these are the
failure modes of its MI355X restatement).

* A target sort that flags an error is re-run, and the registration goes on: forced here by launching fewer radix passes
  than the key needs (ndt_set_build_options(radix_passes=1): the last launched pass flags it), which takes the same
  path as a decoupled look-back that timed out (the ticket-ordered re-run is checked through tile_tickets=1) — grid and
  align bit-identical to an unforced ctx.
* The radix passes a target sort launches follow the previous grid's key width (C2's 23-bit keys: three, no empty fourth).
* The align-graph cache (64 chains) cycled through more than 64 source-size buckets on one ctx while getFitnessScore's
  side lane runs beside every align: every result equals a fresh ctx's.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

xa = pytest.importorskip("xchu_slam_amd")
from helpers import small_pair  # noqa: E402


def _ctx(pair, **opts):
    g = xa.NormalDistributionsTransform()
    g.setResolution(1.0)
    g.setTransformationEpsilon(0.0)
    g.setMaximumIterations(8)
    if opts:
        g.set_build_options(**opts)
    g.setInputTarget(pair.target)
    g.setInputSource(pair.source)
    return g


def _same_grid(a, b):
    assert a.grid_info() == b.grid_info()
    la, lb = a.grid_leaves(), b.grid_leaves()
    for k in ("keys", "npts", "mean", "icov", "centroid"):
        assert np.array_equal(la[k], lb[k]), k


def test_flagged_build_is_rerun_by_the_align():
    """Too few radix passes (forced): the align finds the flag in its read-back, re-runs the build with four passes and
    the align itself — the result is bitwise an unforced ctx's."""
    pair = small_pair(seed=5, half=60.0, n_source=6000)
    ref = _ctx(pair)
    ref.align(pair.guess, want_output=False)
    r0 = ref.result()
    f = _ctx(pair, radix_passes=1)
    assert f.build_stats()["radix_passes"] == 1
    f.align(pair.guess, want_output=False)
    r1 = f.result()
    st = f.build_stats()
    assert st["rerun"] == 1 and st["rerun_lookback"] == 0 and st["tile_tickets"] == 0, st
    assert np.array_equal(r0["final_tf"], r1["final_tf"]) and r0["n_pairs"] == r1["n_pairs"]
    for a, b in zip(ref.history(), f.history()):
        assert np.array_equal(a["x"], b["x"]) and a["pairs"] == b["pairs"]
    _same_grid(ref, f)
    # a synchronous grid reader (no align in between) re-runs a flagged build too
    f.setInputTarget(pair.target)
    _same_grid(ref, f)
    assert f.build_stats()["rerun"] == 2
    ref.close()
    f.close()


def test_ticket_ordered_build_matches():
    """The mode a look-back timeout switches a ctx to (tiles by atomic ticket in every radix pass and scan): the same
    grid and the same registration, bit for bit."""
    pair = small_pair(seed=6, half=60.0, n_source=6000)
    ref = _ctx(pair)
    t = _ctx(pair, tile_tickets=True)
    assert t.build_stats()["tile_tickets"] == 1
    _same_grid(ref, t)
    for g in (ref, t):
        g.align(pair.guess, want_output=False)
    assert np.array_equal(ref.getFinalTransformation(), t.getFinalTransformation())
    assert t.build_stats()["rerun"] == 0
    ref.close()
    t.close()


def test_ticket_mode_after_default_builds():
    """A ctx switched to ticket-ordered tiles after default builds (what a look-back timeout does mid-life): the scans'
    ticket base must follow the device counter, which only ticket-mode launches advance — a base counted over every
    launch gave negative tiles (round-6 C4 at 16 queues x 8 streams: registrations off by ~0.15 m on the switched
    contexts).  Grids and aligns bit-identical to a default ctx, over several builds in each mode."""
    pair = small_pair(seed=9, half=60.0, n_source=6000)
    ref = _ctx(pair)
    ref.align(pair.guess, want_output=False)
    g = _ctx(pair)
    g.align(pair.guess, want_output=False)
    g.setInputTarget(pair.target)
    g.align(pair.guess, want_output=False)
    g.set_build_options(tile_tickets=True)
    for _ in range(3):
        g.setInputTarget(pair.target)
        _same_grid(ref, g)
        g.align(pair.guess, want_output=False)
        assert np.array_equal(ref.getFinalTransformation(), g.getFinalTransformation())
    assert g.build_stats()["tile_tickets"] == 1 and g.build_stats()["rerun"] == 0
    ref.close()
    g.close()


def test_radix_passes_follow_key_width():
    """After a grid of <= 23-bit keys (a ~200 m box at 1 m) the next target sort launches three radix passes; a
    forced count overrides it (test hook), 0 restores the prediction."""
    pair = small_pair(seed=7, half=60.0, n_source=4000)
    g = _ctx(pair)
    assert g.build_stats()["radix_passes"] == 4  # nothing read back yet
    g.align(pair.guess, want_output=False)
    info = g.grid_info()
    cells = int(np.prod(info["div_b"]))
    bits = int(cells - 1).bit_length()
    assert g.build_stats()["radix_passes"] == min(4, (bits + 1 + 7) // 8)
    g.set_build_options(radix_passes=2)
    assert g.build_stats()["radix_passes"] == 2
    g.set_build_options(radix_passes=0)
    assert g.build_stats()["radix_passes"] == min(4, (bits + 1 + 7) // 8)
    g.close()


def test_graph_cache_cycles_with_side_lane_busy():
    """70 source sizes of distinct launch buckets (more than the 64 cached chains, so entries are evicted while the
    stream may still hold work) through one ctx, each align followed by an asynchronous getFitnessScore on the fit lane
    that runs beside the next align; every align equals a fresh ctx's align of the same cloud."""
    pair = small_pair(seed=8, half=60.0, n_source=14000)
    g = _ctx(pair)
    lib = g._lib
    sizes = [4200 + 130 * i for i in range(70)]
    check_at = {0, 33, 64, 69}
    pending = False
    for i, n in enumerate(sizes):
        src = pair.source[:n]
        g.setInputSource(src)
        g.align(pair.guess, want_output=False)
        if pending:
            out = C.c_double()
            xa._lib.check(lib.ndt_fitness_score_result(g.ctx, C.byref(out)), g.ctx)
            assert np.isfinite(out.value)
        xa._lib.check(lib.ndt_fitness_score_async(g.ctx, None, C.c_double(np.finfo(np.float64).max)), g.ctx)
        pending = True
        if i in check_at:
            T = g.getFinalTransformation()
            f = _ctx(pair)
            f.setInputSource(src)
            f.align(pair.guess, want_output=False)
            assert np.array_equal(T, f.getFinalTransformation()), (i, n)
            f.close()
    out = C.c_double()
    xa._lib.check(lib.ndt_fitness_score_result(g.ctx, C.byref(out)), g.ctx)
    g.close()
