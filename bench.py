"""NDT scan-matching benchmark (BASELINE.json metric) on MI355X.

One step = one scan->localmap registration exactly as odom_node performs it per scan
(odom_node.cpp:227-283, 348-349): setInputTarget (device voxel-covariance build of the localmap points)
+ setInputSource + align (30 max iterations, trans_eps 0 => fixed work: 1 + 32 derivative passes).
Workload (BASELINE configs[1] / SURVEY §8d C2): a 120k-point LiDAR-like scan against a localmap of ~1.92M
points = ~200k valid 1 m voxels, DIRECT7, synthetic (seeded world, no KITTI data on the box).
Inputs are resident in HBM before the timed region.  N GPUs: one process per GPU, each rank registers its
own independent pairs (weak scaling, batched offline replay); results are gathered once.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "NDT scans/sec (120k-pt scan vs 200k-voxel localmap, 30 iters) at 1/2/4/8 GPUs; % HBM BW"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
MAX_ITER = 30
# SURVEY §8d configs.  c2 is the default (the configuration BASELINE's metric is quoted on); c5 is the dense
# stress case on which the HBM-bandwidth target is judged (1M-pt scan vs ~2M voxels of ~8 points at 0.5 m).
WORKLOADS = {
    "c2": dict(desc="C2: single 120k-pt scan vs ~200k-voxel localmap per step (target build + align), BASELINE configs[1]",
               half=210.0, density=8.0, n_source=120_000, resolution=1.0, max_range=60.0, pairs=4),
    "c5": dict(desc="C5 dense stress: 1M-pt scan vs ~2M-voxel localmap at res 0.5 per step (target build + align), "
                    "BASELINE configs[4]",
               half=330.0, density=32.0, n_source=1_000_000, resolution=0.5, max_range=80.0, pairs=1),
    "c3": dict(desc="C3 replay: synthetic 120k-pt scans at consecutive KITTI-00 GT poses streamed through the native "
                    "odom_node scan loop (constant-velocity guess, 0.5 m keyframes, 1.0 m localmap downsample, 5 m "
                    "localmap reset, getFitnessScore per scan); odom_node defaults except ndt_resolution 1.0",
               n_source=120_000, resolution=1.0, max_range=60.0, scans=4541),
    "c4": dict(desc="C4 batched offline replay: independent pairs (120k-pt scan vs ~200k-voxel localmap, target build + align "
                    "each, 30 iters) registered through ndt_align_batch with NDT_BATCH_STREAMS streams per GPU (default 2); "
                    "ranks take disjoint pairs (SURVEY 8e)",
               half=210.0, density=8.0, n_source=120_000, resolution=1.0, max_range=60.0, pairs=4),
    "fe": dict(desc="filter_node front end (SURVEY 8f row 4): raw 120k-point HDL-64-like scan (out to 80 m, NaNs, outliers) -> "
                    "NaN removal, 1 < r < 60 m crop, VoxelGrid 0.5 m, StatisticalOutlierRemoval(30, 1.0) -> /filtered_points",
               n_raw=120_000, pairs=4),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_pool(rank: int, n_pairs: int, wl: dict):
    from xchu_slam_amd import synth
    pool = []
    for i in range(n_pairs):
        seed = 1000 * rank + 17 * i + 1
        w = synth.make_world(seed, half=wl["half"])
        pool.append(synth.make_pair(w, wl["density"], wl["n_source"], seed=seed + 3, max_range=wl["max_range"]))
    return pool


def cpu_info():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model


def cpu_baseline(pair, budget_s: float = 25.0, resolution: float = 1.0):
    """Time the oracle (CPU restatement of ndt_omp, test infrastructure) on the same workload.

    Sample: full registrations (target build + align) of the first pool pair with all host threads
    available to this process (OMP_NUM_THREADS), then one with 1 thread (as wired in odom_node.cpp:74),
    bounded by `budget_s` of CPU work."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or 1))
    res = {}
    for nt in (threads, 1):
        o = oracle_lib.OracleNDT(num_threads=nt, resolution=resolution, step_size=0.1, trans_eps=0.0, max_iter=MAX_ITER)
        times = []
        t_start = time.perf_counter()
        while True:
            t0 = time.perf_counter()
            o.set_target(pair.target)
            o.set_source(pair.source)
            r = o.align(pair.guess)
            times.append(time.perf_counter() - t0)
            if time.perf_counter() - t_start > budget_s / 2 or len(times) >= 3:
                break
        o.close()
        res[nt] = (float(np.median(times)), len(times), r)
    t_all, n_all, _ = res[threads]
    t_one, n_one, _ = res[1]
    return {
        "value": 1.0 / t_all,
        "unit": "scans/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{n_all} full registration(s) (voxel build of {len(pair.target)} pts + align of {len(pair.source)} pts, "
                   f"{MAX_ITER} iters) with {threads} OpenMP threads, median; oracle = CPU restatement of ndt_omp "
                   f"(std::map leaves, DIRECT7, f32 pair math, -O2) on '{cpu_info()}'"),
        "value_1thread": 1.0 / t_one,
        "sample_1thread": f"{n_one} registration(s), 1 thread (odom_node.cpp:74 wiring)",
    }


def _c3_chunk(args):
    """Worker: sensor-frame scans k0..k1 of the C3 sequence (float32 (N,3) each)."""
    k0, k1, n_points, seed = args
    from xchu_slam_amd import synth
    tum = np.load(os.path.join(ROOT, "tests", "golden", "kitti00_gt.npz"))["tum"]
    poses = synth.kitti_poses(tum)
    world = c3_world(tum, seed)
    return [synth.sensor_scan(world, poses[k], n_points, seed + 7919 * (k + 1)) for k in range(k0, k1)]


def c3_world(tum, seed):
    from xchu_slam_amd import synth
    xy = synth.kitti_poses(tum)[:, :2, 3]
    return synth.make_street_world(seed, xy, float(np.abs(xy).max()) + 90.0)


def make_c3_scans(n_scans: int, n_points: int, seed: int = 0, workers: int = 0):
    """C3 inputs: scans at KITTI-00 GT poses 0..n_scans-1, generated in parallel host workers."""
    import multiprocessing as mp
    workers = workers or max(1, min(16, (os.cpu_count() or 2) - 1))
    step = max(1, -(-n_scans // (workers * 4)))
    jobs = [(k, min(n_scans, k + step), n_points, seed) for k in range(0, n_scans, step)]
    if workers == 1 or len(jobs) == 1:
        parts = [_c3_chunk(j) for j in jobs]
    else:
        with mp.get_context("spawn").Pool(workers) as pool:
            parts = pool.map(_c3_chunk, jobs)
    return [s for p in parts for s in p]


def cpu_baseline_c3(scans, budget_s: float, resolution: float):
    """Time the CPU restatement of the scan loop (oracle registration, tests/odom_restate.py) on the first scans."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import odom_restate
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or 1))
    o = odom_restate.OdomRestatement(ndt_resolution=resolution, num_threads=threads)
    t0 = time.perf_counter()
    n = 0
    for s in scans:
        o.process(s)
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    el = time.perf_counter() - t0
    o.close()
    return {"value": n / el, "unit": "scans/s", "cores": threads, "kind": "port",
            "sample": (f"first {n} scans of the C3 replay through the CPU restatement of odom_node's scan loop (oracle "
                       f"ndt_omp restatement, DIRECT7, {threads} OpenMP threads; no getFitnessScore) on '{cpu_info()}'")}


def run_c3(args, wl):
    """C3: the whole replay is one timed run; a step is one scan through OdomEstimate."""
    import xchu_slam_amd as xa
    n_scans = args.steps if args.steps_given else wl["scans"]
    t0 = time.perf_counter()
    scans = make_c3_scans(n_scans + args.warmup, wl["n_source"])
    log(f"generated {len(scans)} C3 scans in {time.perf_counter() - t0:.1f}s")
    # warmup: a separate driver over the first scans (JIT/alloc), then the measured replay from scan 0
    warm = xa.LidarOdom(ndt_resolution=wl["resolution"])
    for k in range(args.warmup):
        warm.process(scans[k], 0.1 * k)
    warm.close()
    odom = xa.LidarOdom(ndt_resolution=wl["resolution"])
    dev = [odom.upload(s) for s in scans[:n_scans]]
    lib = odom._lib
    lib.ndt_synchronize(odom._ctx)
    odom.set_profiling(True)
    t_start = time.perf_counter()
    recs = []
    for k, (ptr, n) in enumerate(dev):
        recs.append(odom.process_device(ptr, n, 0.1 * k))
    lib.ndt_synchronize(odom._ctx)
    elapsed = time.perf_counter() - t_start
    tm = odom.timings()
    from xchu_slam_amd import synth
    tum = np.load(os.path.join(ROOT, "tests", "golden", "kitti00_gt.npz"))["tum"]
    poses = synth.kitti_poses(tum, count=n_scans)
    P0 = np.linalg.inv(poses[0])
    ape = [float(np.linalg.norm(r["t_localizer"][:3, 3].astype(np.float64) - (P0 @ poses[k])[:3, 3])) for k, r in enumerate(recs)]
    odom.close()
    if args.save_traj:
        np.savez(args.save_traj, t_localizer=np.stack([r["t_localizer"] for r in recs]), gt=np.stack([P0 @ p for p in poses]),
                 iters=np.array([r["final_num_iteration"] for r in recs]), n_localmap=np.array([r["n_localmap"] for r in recs]),
                 ms=np.array([[r[k] for k in ("ms_align", "ms_fitness", "ms_map", "ms_total")] for r in recs]),
                 fitness=np.array([r["fitness_score"] for r in recs]))
    value = n_scans / elapsed
    achieved = (tm["pass_bytes_avg"] / (tm["ms_pass_avg"] * 1e-3) / 1e9) if tm["ms_pass_avg"] > 0 else 0.0
    line = {
        "metric": METRIC, "value": round(value, 3), "unit": "scans/s", "n_gpus": 1, "steps": n_scans, "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / n_scans, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32 (f64 accumulate)",
        "data": "synthetic scans (seeded world) at KITTI-00 ground-truth poses (tests/golden/kitti00_gt.npz)",
        "config": {"workload": wl["desc"], "n_source": wl["n_source"], "scans": n_scans, "resolution": wl["resolution"],
                   "keyframes": int(sum(r["keyframe"] for r in recs)), "localmap_resets": int(sum(r["localmap_reset"] for r in recs)),
                   "mean_localmap_points": round(float(np.mean([r["n_localmap"] for r in recs])), 1),
                   "mean_iterations": round(float(np.mean([r["final_num_iteration"] for r in recs])), 3),
                   "search": "DIRECT7", "parallelism": "sequential replay on one GPU (each guess depends on the last pose)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                     "kernel": "k_pass_direct<DIRECT7> (derivative pass)", "ms_per_launch": round(tm["ms_pass_avg"], 5),
                     "algorithmic_bytes_per_launch": round(tm["pass_bytes_avg"])},
        "breakdown_ms_per_step": {k: round(float(np.mean([r[k] for r in recs])), 4)
                                  for k in ("ms_align", "ms_fitness", "ms_map", "ms_total")},
        "ape_m": {"mean": round(float(np.mean(ape)), 4), "max": round(float(np.max(ape)), 4), "final": round(ape[-1], 4)},
        "cpu_baseline": None,
    }
    if not args.no_cpu_baseline:
        try:
            line["cpu_baseline"] = cpu_baseline_c3(scans[:n_scans], args.cpu_budget, wl["resolution"])
            line["vs_cpu"] = round(value / line["cpu_baseline"]["value"], 2)
        except Exception as e:
            log(f"cpu baseline failed: {e!r}")
    print(json.dumps(line), flush=True)


def run_fe(args, wl):
    """Front end: a step = one raw scan through filter_node's /filtered_points pipeline (device-resident input)."""
    import ctypes as C
    import xchu_slam_amd as xa
    from xchu_slam_amd import _lib
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import raw_scan
    n_scans = args.pairs or wl["pairs"]
    scans = [raw_scan(seed=100 + k, n_points=wl["n_raw"], n_outliers=wl["n_raw"] // 200) for k in range(n_scans)]
    ndt = xa.NormalDistributionsTransform()
    lib = ndt._lib
    prm = _lib.FilterParams()
    lib.ndt_filter_default_params(C.byref(prm))
    dev = [(ndt.device_upload(s), len(s)) for s in scans]
    d_out = C.c_void_p()
    lib.ndt_device_alloc(ndt.ctx, max(len(s) for s in scans) * 16, C.byref(d_out))
    nout = C.c_size_t()

    def step(i):
        ptr, n = dev[i % len(dev)]
        _lib.check(lib.ndt_filter_scan_device(ndt.ctx, C.byref(prm), C.c_void_p(ptr), n, d_out, C.byref(nout)), ndt.ctx)
        return nout.value

    for i in range(args.warmup):
        step(i)
    lib.ndt_synchronize(ndt.ctx)
    t0 = time.perf_counter()
    outs = [step(i) for i in range(args.steps)]
    lib.ndt_synchronize(ndt.ctx)
    el = time.perf_counter() - t0
    value = args.steps / el
    line = {"metric": "filter_node front end scans/sec (raw 120k-pt scan -> /filtered_points)", "value": round(value, 3),
            "unit": "scans/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * el / args.steps, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32 (f64 distance sums)", "data": "synthetic raw scans (tests/helpers.raw_scan)",
            "config": {"workload": wl["desc"], "n_raw": wl["n_raw"], "mean_filtered_points": round(float(np.mean(outs)), 1)},
            "cpu_baseline": None}
    if not args.no_cpu_baseline:
        import oracle_lib
        t0 = time.perf_counter()
        k = 0
        while True:
            oracle_lib.filter_scan(scans[k % len(scans)], is_dense=False)
            k += 1
            if time.perf_counter() - t0 > min(args.cpu_budget, 10.0) or k >= 5:
                break
        cpu = k / (time.perf_counter() - t0)
        line["cpu_baseline"] = {"value": round(cpu, 4), "unit": "scans/s", "cores": 1, "kind": "port",
                                "sample": f"{k} scans through the oracle restatement (hash-grid exact k-NN, 1 thread) on '{cpu_info()}'"}
        line["vs_cpu"] = round(value / cpu, 2)
    print(json.dumps(line), flush=True)


def load_pmc_traffic(workload: str):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json" if workload == "c2" else f"pmc_traffic_{workload}.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pairs", type=int, default=0, help="distinct scan/localmap pairs per rank (cycled); 0 = workload default")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=25.0)
    ap.add_argument("--save-traj", default="", help="c3: write the per-scan trajectory / timings (.npz)")
    ap.add_argument("--no-kernel-stamps", action="store_true", help="time without the in-kernel pass stamps (no roofline timing)")
    args = ap.parse_args()
    args.steps_given = any(a == "--steps" or a.startswith("--steps=") for a in sys.argv[1:])
    if args.workload == "c3":
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            raise SystemExit("c3 is a sequential replay on one GPU (SURVEY 8e); run it with --gpus 1")
        return run_c3(args, WORKLOADS["c3"])
    if args.workload == "fe":
        return run_fe(args, WORKLOADS["fe"])

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        tdist.init_process_group(backend=backend)
        dist = tdist

    import xchu_slam_amd as xa
    from xchu_slam_amd import synth

    wl = WORKLOADS[args.workload]
    t0 = time.perf_counter()
    pool = make_pool(rank, args.pairs or wl["pairs"], wl)
    log(f"[rank {rank}] generated {len(pool)} pairs in {time.perf_counter() - t0:.1f}s "
        f"(M={len(pool[0].target)}, N={len(pool[0].source)})")

    ndt = xa.NormalDistributionsTransform(device=local_rank)
    ndt.setNeighborhoodSearchMethod(xa.DIRECT7)
    ndt.setResolution(wl["resolution"])
    ndt.setStepSize(0.1)
    ndt.setTransformationEpsilon(0.0)
    ndt.setMaximumIterations(MAX_ITER)
    dev = []
    for p in pool:
        dt = ndt.device_upload(synth.to_xyz4(p.target))
        ds = ndt.device_upload(synth.to_xyz4(p.source))
        dev.append((dt, len(p.target), ds, len(p.source)))

    def step(i):
        dt, nt, ds, ns = dev[i % len(dev)]
        ndt.setInputTargetDevice(dt, nt)
        ndt.setInputSourceDevice(ds, ns)
        ndt.align(pool[i % len(pool)].guess, want_output=False)
        return ndt.result()

    batched = args.workload == "c4"

    def run_batch(i0, k):
        # C4: k pairs in one ndt_align_batch call (several streams in flight)
        return ndt.align_batch([(dev[i % len(dev)][0], dev[i % len(dev)][1], dev[i % len(dev)][2], dev[i % len(dev)][3],
                                 pool[i % len(pool)].guess) for i in range(i0, i0 + k)])

    if batched:
        run_batch(0, max(args.warmup, 2))
    else:
        for i in range(args.warmup):
            step(i)
    grid = ndt.grid_info()
    ndt.setProfiling(not batched and not args.no_kernel_stamps)

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    ndt._lib.ndt_synchronize(ndt.ctx)
    t_start = time.perf_counter()
    results = []
    ms_build = ms_align = 0.0
    if batched:
        results = run_batch(0, args.steps)
    else:
        for i in range(args.steps):
            r = step(i)
            tm = ndt.timings()
            ms_build += tm["ms_build"]
            ms_align += tm["ms_align"]
            results.append(r)
    ndt._lib.ndt_synchronize(ndt.ctx)
    barrier()
    elapsed = time.perf_counter() - t_start
    tm = ndt.timings()

    # ---- accuracy of this rank's registrations (synthetic ground truth)
    errs = []
    for i, r in enumerate(results[: len(pool)]):
        d = np.linalg.inv(pool[i % len(pool)].true_pose) @ r["final_tf"].astype(np.float64)
        errs.append(float(np.linalg.norm(d[:3, 3])))

    t_max = elapsed
    scans_total = args.steps * world
    if dist is not None:
        import torch
        dev_t = "cuda" if dist.get_backend() == "nccl" else "cpu"
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev_t)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
        # one gather of the per-pair result records (final pose + iterations), SURVEY §8e
        rec = torch.tensor([[*r["final_tf"].reshape(-1).tolist(), r["nr_iterations"], r["n_pairs"]] for r in results],
                           dtype=torch.float64, device=dev_t)
        gathered = [torch.empty_like(rec) for _ in range(world)]
        dist.all_gather(gathered, rec)

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    value = scans_total / t_max
    ms_step = 1000.0 * t_max / args.steps
    achieved = (tm["pass_bytes_avg"] / (tm["ms_pass_avg"] * 1e-3) / 1e9) if tm["ms_pass_avg"] > 0 else 0.0
    traffic = load_pmc_traffic(args.workload)
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "scans/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (f64 accumulate)",
        "data": "synthetic (seeded LiDAR-like world; no KITTI scans on the box)",
        "config": {
            "workload": wl["desc"],
            "n_source": len(pool[0].source),
            "n_target_points": len(pool[0].target),
            "voxels_valid": grid["n_valid"],
            "voxels_cloud": grid["n_cloud"],
            "resolution": wl["resolution"],
            "max_iter": MAX_ITER,
            "trans_eps": 0.0,
            "passes_per_align": results[-1]["n_passes"],
            "search": "DIRECT7",
            "pairs_per_rank": len(pool),
            "parallelism": f"replicas x{world} (independent pairs per GPU)",
        },
        "roofline": {
            "bound": "hbm",
            # null (not 0) when the pass was not timed (batched C4 / --no-kernel-stamps run without the stamps)
            "achieved": round(achieved, 2) if achieved > 0 else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved > 0 else None,
            "traffic": traffic,
            "kernel": "k_pass_direct<DIRECT7> (derivative pass)",
            "ms_per_launch": round(tm["ms_pass_avg"], 5),
            "algorithmic_bytes_per_launch": round(tm["pass_bytes_avg"]),
            "phases_ms": {k: round(v, 5) for k, v in tm["pass_phases_ms"].items()},
            **({k2: {k: round(v, 5) for k, v in tm[k2].items()} for k2 in ("workgroup_phases_ms", "tail_phases_ms")
                if k2 in tm}),
        },
        "breakdown_ms_per_step": {"voxel_build": round(ms_build / args.steps, 4), "align": round(ms_align / args.steps, 4)},
        "mean_translation_error_m": round(float(np.mean(errs)), 4) if errs else None,
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu_baseline:
        try:
            line["cpu_baseline"] = cpu_baseline(pool[0], args.cpu_budget, wl["resolution"])
            line["vs_cpu"] = round(value / line["cpu_baseline"]["value"], 2)
        except Exception as e:  # the GPU number stands on its own
            log(f"cpu baseline failed: {e!r}")
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
