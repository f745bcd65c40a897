"""NDT scan-matching benchmark (BASELINE.json metric) on MI355X.

One step = one scan->localmap registration exactly as odom_node performs it per scan
(odom_node.cpp:227-283, 348-349): setInputTarget (device voxel-covariance build of the localmap points)
+ setInputSource + align (30 max iterations, trans_eps 0 => fixed work: 1 + 32 derivative passes).
Workload (BASELINE configs[1] / SURVEY §8d C2): a 120k-point LiDAR-like scan against a localmap of ~1.92M
points = ~200k valid 1 m voxels, DIRECT7, synthetic (seeded world, no KITTI data on the box).
Inputs are resident in HBM before the timed region.

N GPUs: one process per GPU (launched by torch.distributed.run, or by this script itself when `--gpus N` is given
without a launcher).  c2/c5: each rank registers its own pairs (replicas, weak scaling).  c4: a fixed
set of 4096 pairs sharded contiguously over the ranks (strong scaling).  Per-registration result records are gathered
once at the end (xchu_slam_amd/batch.py; RCCL over xGMI when the group is nccl).
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
    "c4": dict(desc="C4 batched offline replay: a fixed set of independent pairs (pair i: ~1.9M-pt localmap of a world seeded "
                    "1000+i = ~200k valid 1 m voxels, 120k-pt scan seeded 5000+i; target build + align each, 30 iters) sharded "
                    "contiguously over the GPUs, registered through ndt_align_batch (three HIP streams per GPU, "
                    "default 3)",
               half=210.0, density=8.0, n_source=120_000, resolution=1.0, max_range=60.0, pairs_total=4096),
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


def _oracle_env(threads: int) -> None:
    """BASELINE.md §3 / SURVEY §8d: OpenMP bound close to cores.  libgomp reads these when it initialises, i.e. when
    the oracle library is first loaded, so they are set before that (the product library does not use OpenMP)."""
    os.environ.setdefault("OMP_PROC_BIND", "close")
    os.environ.setdefault("OMP_PLACES", "cores")
    os.environ["OMP_NUM_THREADS"] = str(threads)


def host_threads() -> int:
    """Every CPU this process may run on (its affinity mask; recorded in core_counts)."""
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        return max(1, os.cpu_count() or 1)


def share_threads() -> int:
    """Threads of the CPU baseline's all-core legs (BASELINE.md §3 "all cores"; the class default omp_get_max_threads(),
    ndt_omp_impl.hpp:68, reads OMP_NUM_THREADS): the host's CPU share as the box announces it (OMP_NUM_THREADS, 16 per
    GPU on the GPU box), capped at the affinity count.  The GPU box's affinity mask is the whole shared machine (256
    CPUs): 256 oracle threads there ran 0.18 scans/s against 0.93 with 16 (other tenants' work on the same cores), so
    the share, not the mask, is the box's "all cores"."""
    t = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(t, host_threads())) if t > 0 else host_threads()


def core_counts() -> dict:
    return {"affinity": host_threads(), "box_cpus": os.cpu_count(), "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(target, source, guess, budget_s: float = 40.0, resolution: float = 1.0):
    """Time the oracle (CPU restatement of ndt_omp, test infrastructure) on the same workload, BASELINE.md §3 protocol:
    OMP_PROC_BIND=close OMP_PLACES=cores, 1 warm-up then >= 5 samples (median) of setInputTarget and of
    setInputSource + align, timed separately; all host threads (the class default, ndt_omp_impl.hpp:68) with the
    -O2 build (the reference .so: GCC, SSE only) and the -O3 -march=x86-64-v3 build, plus 1 thread (odom_node.cpp:74).
    Bounded by `budget_s` of wall time: a leg that runs out of budget reports the samples it has (>= 1)."""
    threads = share_threads()
    env_counts = core_counts()
    _oracle_env(threads)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib

    t_begin = time.perf_counter()

    def leg(variant, nt, share):
        o = oracle_lib.OracleNDT(variant=variant, num_threads=nt, resolution=resolution, step_size=0.1, trans_eps=0.0,
                                 max_iter=MAX_ITER)
        t_leg = time.perf_counter()
        tt, ta = [], []
        for k in range(6):  # sample 0 = warm-up
            t0 = time.perf_counter()
            o.set_target(target)
            t1 = time.perf_counter()
            o.set_source(source)
            o.align(guess)
            t2 = time.perf_counter()
            if k > 0:
                tt.append(t1 - t0)
                ta.append(t2 - t1)
            if k > 0 and time.perf_counter() - t_leg > share:
                break
        o.close()
        if not tt:  # the warm-up alone used the budget: report it
            tt, ta = [t1 - t0], [t2 - t1]
        mt, ma = float(np.median(tt)), float(np.median(ta))
        return {"scans_per_s": round(1.0 / (mt + ma), 5), "set_target_ms": round(1e3 * mt, 2), "align_ms": round(1e3 * ma, 2),
                "samples": len(tt), "threads": nt, "build": "-O2 (SSE)" if variant == "" else "-O3 -march=x86-64-v3"}

    legs = {"all_O2": leg("", threads, 0.3 * budget_s), "all_v3": leg("_v3", threads, 0.25 * budget_s)}
    legs["one_O2"] = leg("", 1, max(1.0, budget_s - (time.perf_counter() - t_begin)))
    head = legs["all_O2"]
    return {
        "value": head["scans_per_s"],
        "unit": "scans/s",
        "cores": threads,
        "core_counts": env_counts,
        "kind": "port",
        "sample": (f"median of {head['samples']} full registrations after 1 warm-up (setInputTarget {head['set_target_ms']} ms: "
                   f"voxel build of {len(target)} pts; align {head['align_ms']} ms: {len(source)} pts, {MAX_ITER} iters) with "
                   f"{threads} OpenMP threads (OMP_PROC_BIND={os.environ.get('OMP_PROC_BIND')}, "
                   f"OMP_PLACES={os.environ.get('OMP_PLACES')}); oracle = CPU restatement of ndt_omp (std::map leaves, DIRECT7, "
                   f"f32 pair math, -O2) on '{cpu_info()}'"),
        "legs": legs,
        "value_1thread": legs["one_O2"]["scans_per_s"],
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
        # close() + join() rather than the context exit's terminate(): the workers end on their own (a profiled run
        # would otherwise record their SIGTERM as aborts)
        pool = mp.get_context("spawn").Pool(workers)
        try:
            parts, t0 = [], time.perf_counter()
            for k, part in enumerate(pool.imap(_c3_chunk, jobs)):
                parts.append(part)
                if k % max(1, len(jobs) // 8) == 0:
                    log(f"C3 scans: {sum(len(p) for p in parts)}/{n_scans} generated ({time.perf_counter() - t0:.0f}s)")
            pool.close()
        except BaseException:
            pool.terminate()
            raise
        finally:
            pool.join()
    return [s for p in parts for s in p]


def cpu_baseline_c3(scans, budget_s: float, resolution: float):
    """Time the CPU restatement of the scan loop (oracle registration, tests/odom_restate.py) on the first scans."""
    threads = share_threads()
    _oracle_env(threads)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import odom_restate
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
    return {"value": n / el, "unit": "scans/s", "cores": threads, "core_counts": core_counts(), "kind": "port",
            "sample": (f"first {n} scans of the C3 replay through the CPU restatement of odom_node's scan loop (oracle "
                       f"ndt_omp restatement, DIRECT7, {threads} OpenMP threads; no getFitnessScore) on '{cpu_info()}'")}


def run_c3(args, wl):
    """C3: the whole replay is one timed run; a step is one scan through OdomEstimate."""
    import xchu_slam_amd as xa
    n_scans = min(args.steps if args.steps_given else wl["scans"], wl["scans"])  # KITTI-00 has 4541 poses
    t0 = time.perf_counter()
    # the warm-up driver replays the first scans (then discarded); the measured replay starts again at scan 0
    scans = make_c3_scans(max(n_scans, args.warmup), wl["n_source"])
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
    # the whole sequence through the pipelined replay entry point (ndt_odom_process_batch_device: a scan's fitness
    # score and keyframe insertion are collected after the next scan's align; records identical to per-scan calls,
    # tests/test_gpu_c3_fullsize.py)
    stamps = [0.1 * k for k in range(len(dev))]
    t_start = time.perf_counter()
    recs = odom.process_batch_device(dev, stamps)
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
                     **pass_kernel_desc(tm), "ms_per_launch": round(tm["ms_pass_avg"], 5),
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




def pass_kernel_desc(tm: dict) -> dict:
    """Name and timing of the derivative-pass kernel the align ran: the leading-tail chain (k_pass_lead: a pass's kernel
    runs the previous pass's Newton step, then its own body; stamped at workgroup 0's start, pass = start to the next
    kernel's start) or the last-workgroup tails (k_pass_direct: workgroup 0's kernel entry, stamped before anything else,
    to the end of the last workgroup's tail, with phases)."""
    if any(tm.get("pass_phases_ms", {}).values()):
        return {"kernel": "k_pass_direct<DIRECT7> (derivative pass + last-workgroup Newton step)",
                "timing": "in-kernel s_memrealtime stamps (workgroup 0's kernel entry -> end of the last workgroup's tail) over "
                          "the timed steps",
                "phases_ms": {k: round(v, 5) for k, v in tm["pass_phases_ms"].items()}}
    return {"kernel": "k_pass_lead<DIRECT7> (previous pass's Newton step in every workgroup + derivative pass body)",
            "timing": "in-kernel s_memrealtime stamps (workgroup 0's start of a pass -> of the next pass, launch gap "
                      "included) over the timed steps"}


def load_pmc_traffic(workload: str):
    """HBM bytes per pass launch from the committed rocprofv3 --pmc pass of the same workload (FETCH_SIZE/WRITE_SIZE, the
    gfx950 correction of MI355X_MICROARCH.md); counters cannot be collected inside this timed run.  (bytes, source)."""
    name = "pmc_traffic.json" if workload == "c2" else f"pmc_traffic_{workload}.json"
    path = os.path.join(ROOT, "profiles", name)
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch"), f"profiles/{name} (separate rocprofv3 --pmc run: {d.get('source', 'see file')})"
    except (OSError, ValueError):
        return None, None


# ----------------------------------------------------------------------------------------------- ranks
def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n: int, argv, script: str | None = None, stdout=None, extra_env=None) -> int:
    """`bench.py --gpus N` without a launcher: N child processes, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N,
    MASTER_ADDR 127.0.0.1), as torch.distributed.run would start them.  The parent never touches the GPU (no HIP call,
    no torch.cuda) and exits with the worst child status; if one rank fails the others are stopped."""
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        env.update(extra_env or {})
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__), *argv], env=env,
                                      stdout=stdout if r == 0 else None))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0:
                rc = rc or code
                for q in pending:  # one rank died: the collectives of the others would hang
                    q.terminate()
        time.sleep(0.05)
    return rc


class Dist:
    """One process per GPU (torch.distributed over RCCL when the GPU is visible, gloo on CPU)."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        self.device = None
        if "WORLD_SIZE" in os.environ:  # launched (torch.distributed.run or spawn_ranks): a process group even at world 1
            # torch before libndt_hip.so: torch's libamdhip64 (same soname) then serves both, one HIP runtime per process
            import torch
            import torch.distributed as tdist
            backend = "nccl" if torch.cuda.is_available() else "gloo"
            if backend == "nccl":
                torch.cuda.set_device(self.local_rank)
                self.device = torch.device("cuda", self.local_rank)
            tdist.init_process_group(backend=backend)
            self.dist = tdist

    def barrier(self):
        if self.dist is not None and self.world > 1:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


# ----------------------------------------------------------------------------------------------- c2 / c5 replicas
def run_replicas(args, wl, dd: Dist):
    """c2 / c5: every rank registers its own pairs (replicas, weak scaling); a step = one registration."""
    import xchu_slam_amd as xa
    from xchu_slam_amd import _lib, batch, synth

    rank, world = dd.rank, dd.world
    t0 = time.perf_counter()
    pool = make_pool(rank, args.pairs or wl["pairs"], wl)
    log(f"[rank {rank}] generated {len(pool)} pairs in {time.perf_counter() - t0:.1f}s "
        f"(M={len(pool[0].target)}, N={len(pool[0].source)})")

    ndt = xa.NormalDistributionsTransform(device=dd.local_rank)
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

    # profiling set before the warm-up so that each pool pair's captured chain (profiling is part of the graph key) is
    # built untimed; every pair is registered at least once; the statistics are reset afterwards (no graph rebuild)
    ndt.setProfiling(not args.no_kernel_stamps)
    for i in range(max(args.warmup, len(dev))):
        step(i)
    grid = ndt.grid_info()
    ndt.setProfiling(not args.no_kernel_stamps)

    # The timed loop calls the same C-ABI entry points as step() (setInputTarget -> setInputSource -> align, one
    # registration after the other, each align waited for) with its arguments prepared beforehand, and turns the
    # result structs into dicts after the timed region: the GPU idles while the host runs Python between one align's
    # return and the next target build's first launch, and odom_node's C++ caller has no such per-scan overhead.
    import ctypes as C
    lib, ctx = ndt._lib, ndt.ctx
    f_tgt, f_src, f_align, f_tim = lib.ndt_set_target_device, lib.ndt_set_source_device, lib.ndt_align, lib.ndt_last_timings
    args_tgt = [(C.c_void_p(dt), nt) for dt, nt, _, _ in dev]
    args_src = [(C.c_void_p(ds), ns) for _, _, ds, ns in dev]
    guesses = [np.ascontiguousarray(np.asarray(p.guess, np.float32).T).reshape(-1) for p in pool]
    g_ptrs = [g.ctypes.data_as(C.POINTER(C.c_float)) for g in guesses]
    res_t = type(ndt._result)
    raw = [res_t() for _ in range(args.steps)]
    t_b = [C.c_double() for _ in range(args.steps)]
    t_a = [C.c_double() for _ in range(args.steps)]
    t_p, t_by = C.c_double(), C.c_double()
    npool = len(dev)

    dd.barrier()
    lib.ndt_synchronize(ctx)
    t_start = time.perf_counter()
    for i in range(args.steps):
        k = i % npool
        st = f_tgt(ctx, args_tgt[k][0], args_tgt[k][1], 1) or f_src(ctx, args_src[k][0], args_src[k][1]) or \
            f_align(ctx, g_ptrs[k], C.byref(raw[i])) or f_tim(ctx, C.byref(t_b[i]), C.byref(t_a[i]), C.byref(t_p), C.byref(t_by))
        if st:
            _lib.check(st, ctx)
    lib.ndt_synchronize(ctx)
    dd.barrier()
    elapsed = time.perf_counter() - t_start
    ms_build, ms_align = float(sum(x.value for x in t_b)), float(sum(x.value for x in t_a))
    results = []
    for i in range(args.steps):
        ndt._result = raw[i]
        results.append(ndt.result())
    tm = ndt.timings()

    errs = []
    for i, r in enumerate(results[: len(pool)]):
        d = np.linalg.inv(pool[i % len(pool)].true_pose) @ r["final_tf"].astype(np.float64)
        errs.append(float(np.linalg.norm(d[:3, 3])))

    t_max = dd.max(elapsed)
    # one gather of every rank's per-step result records (RCCL when the group is nccl)
    recs = np.stack([batch.result_record(r) for r in results])
    table = batch.gather_records(recs, args.steps * world, dd.dist, dd.device)
    if rank != 0:
        dd.close()
        return 0

    value = args.steps * world / t_max
    achieved = (tm["pass_bytes_avg"] / (tm["ms_pass_avg"] * 1e-3) / 1e9) if tm["ms_pass_avg"] > 0 else 0.0
    traffic, traffic_src = load_pmc_traffic(args.workload)
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "scans/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * t_max / args.steps, 4),
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
            "registrations_gathered": int(len(table)),
            "parallelism": f"replicas x{world} (independent pairs per GPU, one process per GPU)",
        },
        "roofline": {
            "bound": "hbm",
            # null (not 0) when the pass was not timed (--no-kernel-stamps)
            "achieved": round(achieved, 2) if achieved > 0 else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved > 0 else None,
            "traffic": traffic,
            "traffic_source": traffic_src,
            **pass_kernel_desc(tm),
            "ms_per_launch": round(tm["ms_pass_avg"], 5),
            "algorithmic_bytes_per_launch": round(tm["pass_bytes_avg"]),
            **({k2: {k: round(v, 5) for k, v in tm[k2].items()} for k2 in ("workgroup_phases_ms", "tail_phases_ms")
                if k2 in tm}),
        },
        "breakdown_ms_per_step": {"voxel_build": round(ms_build / args.steps, 4), "align": round(ms_align / args.steps, 4)},
        "mean_translation_error_m": round(float(np.mean(errs)), 4) if errs else None,
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu_baseline:
        try:
            p = pool[0]
            line["cpu_baseline"] = cpu_baseline(p.target, p.source, p.guess, args.cpu_budget, wl["resolution"])
            line["vs_cpu"] = round(value / line["cpu_baseline"]["value"], 2)
        except Exception as e:  # the GPU number stands on its own
            log(f"cpu baseline failed: {e!r}")
    print(json.dumps(line), flush=True)
    dd.close()
    return 0


# ----------------------------------------------------------------------------------------------- c4 batched replay
class GpuC4Backend:
    """C4 pairs on this rank's GPU: generated on the device from their seeds (libndt_synth.so, before the timed region)
    and kept resident in HBM (4096 pairs x ~30 MB = ~125 GB at 1 GPU: fits the MI355X's 288 GB), registered through
    ndt_align_batch (several streams in flight)."""

    def __init__(self, dd: Dist, wl: dict):
        import xchu_slam_amd as xa
        self.wl = wl
        self.device = dd.local_rank
        self.ndt = xa.NormalDistributionsTransform(device=self.device)
        self.ndt.setNeighborhoodSearchMethod(xa.DIRECT7)
        self.ndt.setResolution(wl["resolution"])
        self.ndt.setStepSize(0.1)
        self.ndt.setTransformationEpsilon(0.0)
        self.ndt.setMaximumIterations(MAX_ITER)
        self.pairs = {}
        self.specs = {}

    def prepare(self, indices):
        import ctypes as C
        from xchu_slam_amd import synth
        from xchu_slam_amd._lib import check
        lib, ctx, wl = self.ndt._lib, self.ndt.ctx, self.wl
        d_world = C.c_void_p()
        check(lib.ndt_device_alloc(ctx, 65536 * 4, C.byref(d_world)), ctx)
        for i in indices:
            spec = synth.c4_pair_spec(i, half=wl["half"], density=wl["density"], n_source=wl["n_source"],
                                      max_range=wl["max_range"])
            assert len(spec.world_floats) <= 65536
            ptr = C.c_void_p()
            check(lib.ndt_device_alloc(ctx, (spec.n_target + spec.n_source) * 16, C.byref(ptr)), ctx)
            dt = ptr.value
            ds = dt + spec.n_target * 16
            synth.generate_pair_device(spec, self.device, d_world.value, dt, ds)
            self.pairs[i] = (dt, spec.n_target, ds, spec.n_source, spec.guess)
            self.specs[i] = spec
        check(lib.ndt_device_free(ctx, d_world), ctx)

    def run(self, indices):
        return self.ndt.align_batch([self.pairs[i] for i in indices])

    def synchronize(self):
        self.ndt._lib.ndt_synchronize(self.ndt.ctx)

    def true_pose(self, i):
        return self.specs[i].true_pose

    def host_pair(self, i):
        """(target, source, guess) of pair i copied back to the host (CPU baseline input)."""
        import ctypes as C
        dt, nt, ds, ns, g = self.pairs[i]
        t = np.empty((nt, 4), np.float32)
        s = np.empty((ns, 4), np.float32)
        lib = self.ndt._lib
        lib.ndt_memcpy_d2h(self.ndt.ctx, t.ctypes.data_as(C.c_void_p), C.c_void_p(dt), t.nbytes)
        lib.ndt_memcpy_d2h(self.ndt.ctx, s.ctypes.data_as(C.c_void_p), C.c_void_p(ds), s.nbytes)
        return t[:, :3].copy(), s[:, :3].copy(), g

    def describe(self):
        return {"pair_generation": "on device from the seeds (libndt_synth.so, csrc/synth_pairs.hip), before timing",
                "aligner": "libndt_hip.so ndt_align_batch"}

    def build_stats(self):
        return self.ndt.build_stats()

    def set_profiling(self, on: bool):
        self.ndt.setProfiling(on)

    def timings(self) -> dict:
        return self.ndt.timings()


def c4_roofline(tm, pass_bytes: float, t_max: float):
    """C4 roofline of the derivative pass kernel (k_pass_direct: the batched replay keeps last-workgroup tails so that
    the other streams' bodies fill the CUs a tail leaves idle).  `achieved` = the algorithmic bytes of one launch
    (16 N + 36 P) / its in-kernel duration, averaged over every pass of every stream — with three registrations in flight
    the launches share the GPU, so this is a per-launch lower bound; `aggregate_achieved` = all passes' algorithmic bytes
    of the whole job / the job's wall time (every rank), i.e. the pass bytes the GPUs moved per second, builds included
    in the time."""
    if not tm or tm.get("ms_pass_avg", 0) <= 0:
        return None
    achieved = tm["pass_bytes_avg"] / (tm["ms_pass_avg"] * 1e-3) / 1e9
    agg = pass_bytes / t_max / 1e9 if t_max > 0 else 0.0
    traffic, traffic_src = load_pmc_traffic("c4")
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "traffic_source": traffic_src,
            "kernel": "k_pass_direct<DIRECT7> (derivative pass + last-workgroup Newton step), 3 streams in flight",
            "timing": "in-kernel s_memrealtime stamps (workgroup 0's kernel entry -> end of the last workgroup's tail) of "
                      "every pass of every stream in the timed batch",
            "ms_per_launch": round(tm["ms_pass_avg"], 5), "algorithmic_bytes_per_launch": round(tm["pass_bytes_avg"]),
            "aggregate_achieved": round(agg, 2), "aggregate_frac": round(agg / HBM_PEAK_GBS, 5)}


def run_c4(args, wl, dd: Dist, backend_factory=None):
    """C4 batched offline replay: a FIXED set of `--steps` independent pairs (default 4096) sharded
    contiguously over the ranks (batch.shard_range: 512 per rank at 8 GPUs), no data-path collective, one all-gather of the
    per-pair result records at the end (batch.gather_records; RCCL over xGMI when the group is nccl).  Strong scaling:
    value = all pairs / max-over-ranks time.  A step = one pair (target build + align, 30 iterations)."""
    from xchu_slam_amd import batch
    n_total = args.steps if args.steps_given else wl["pairs_total"]
    mine = list(batch.shard_range(n_total, dd.world, dd.rank))
    backend = (backend_factory or GpuC4Backend)(dd, wl)
    stamps = hasattr(backend, "set_profiling") and not args.no_kernel_stamps
    t0 = time.perf_counter()
    backend.prepare(mine)
    log(f"[rank {dd.rank}] prepared pairs [{mine[0] if mine else 0}, {mine[-1] + 1 if mine else 0}) in "
        f"{time.perf_counter() - t0:.1f}s")
    if stamps:
        backend.set_profiling(True)  # before the warm-up: the stamp flag is part of each captured chain's key
    if mine and args.warmup:
        backend.run(mine[: max(1, min(args.warmup, len(mine)))])  # untimed (allocation, graph capture)
    if stamps:
        backend.set_profiling(True)  # statistics reset (graphs kept)
    backend.synchronize()
    dd.barrier()
    t_start = time.perf_counter()
    results = backend.run(mine) if mine else []
    backend.synchronize()
    dd.barrier()
    elapsed = time.perf_counter() - t_start
    t_max = dd.max(elapsed)
    tm = backend.timings() if stamps else None
    # algorithmic bytes of every derivative pass this rank ran (16 N + 36 P per pass), summed over all ranks
    pass_bytes = float(sum(16.0 * wl["n_source"] * r.get("n_passes", 0) + 36.0 * r.get("n_pairs", 0) for r in results))
    if dd.dist is not None:
        import torch
        tb = torch.tensor([pass_bytes], dtype=torch.float64, device=dd.device)
        dd.dist.all_reduce(tb)
        pass_bytes = float(tb.item())
    local = np.stack([batch.result_record(r) for r in results]) if results else np.zeros((0, batch.RECORD_WIDTH))
    table = batch.gather_records(local, n_total, dd.dist, dd.device)
    errs = [float(np.linalg.norm((np.linalg.inv(backend.true_pose(i)) @ r["final_tf"].astype(np.float64))[:3, 3]))
            for i, r in zip(mine, results)]
    err_stats = np.array([np.mean(errs) if errs else 0.0, np.max(errs) if errs else 0.0, len(errs)])
    if dd.dist is not None:
        import torch
        t = torch.tensor([err_stats[0] * err_stats[2], err_stats[1], err_stats[2]], dtype=torch.float64, device=dd.device)
        parts = [torch.empty_like(t) for _ in range(dd.world)]
        dd.dist.all_gather(parts, t)
        P = np.stack([p.cpu().numpy() for p in parts])
        err_stats = np.array([P[:, 0].sum() / max(P[:, 2].sum(), 1), P[:, 1].max(), P[:, 2].sum()])
    if dd.rank != 0:
        dd.close()
        return 0
    if args.records_out:
        np.save(args.records_out, table)
    value = n_total / t_max
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "scans/s",
        "n_gpus": dd.world,
        "steps": n_total,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * t_max / n_total, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32 (f64 accumulate)",
        "data": "synthetic pairs generated from their seeds (no KITTI scans on the box)",
        "config": {
            "workload": wl["desc"],
            "pairs_total": n_total,
            "pairs_per_rank": [len(batch.shard_range(n_total, dd.world, r)) for r in range(dd.world)],
            "n_source": wl["n_source"],
            "resolution": wl["resolution"],
            "max_iter": MAX_ITER,
            "trans_eps": 0.0,
            "search": "DIRECT7",
            "records_gathered": int(len(table)),
            "converged": int(np.sum(table[:, 17] != 0)) if len(table) else 0,
            "parallelism": f"contiguous pair shards x{dd.world}, one process per GPU, one all-gather of result records",
            **backend.describe(),
        },
        "roofline": c4_roofline(tm, pass_bytes, t_max),
        # rank 0's target builds (ndt_build_stats): re-runs after a flagged sort (look-back timeout / radix width / merge)
        "target_builds": backend.build_stats() if hasattr(backend, "build_stats") else None,
        "mean_translation_error_m": round(float(err_stats[0]), 4),
        "max_translation_error_m": round(float(err_stats[1]), 4),
        "cpu_baseline": None,
    }
    if dd.world == 1 and not args.no_cpu_baseline and mine and hasattr(backend, "host_pair"):
        try:
            t, s, g = backend.host_pair(mine[0])
            line["cpu_baseline"] = cpu_baseline(t, s, g, args.cpu_budget, wl["resolution"])
            line["vs_cpu"] = round(value / line["cpu_baseline"]["value"], 2)
        except Exception as e:
            log(f"cpu baseline failed: {e!r}")
    print(json.dumps(line), flush=True)
    dd.close()
    return 0


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pairs", type=int, default=0, help="c2/c5: distinct scan/localmap pairs per rank (cycled); 0 = default")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=40.0)
    ap.add_argument("--save-traj", default="", help="c3: write the per-scan trajectory / timings (.npz)")
    ap.add_argument("--records-out", default="", help="c4: rank 0 saves the gathered per-pair result table (.npy)")
    ap.add_argument("--no-kernel-stamps", action="store_true", help="time without the in-kernel pass stamps (no roofline timing)")
    argv = sys.argv[1:] if argv is None else argv
    args = ap.parse_args(argv)
    args.steps_given = any(a == "--steps" or a.startswith("--steps=") for a in argv)
    return args, argv


def main(argv=None, c4_backend=None):
    args, argv = parse_args(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    launched = "WORLD_SIZE" in os.environ
    if not launched and args.gpus > 1:
        # no torch.distributed.run around us: start one rank per GPU ourselves (this process stays off the GPU)
        return spawn_ranks(args.gpus, argv, script=os.path.abspath(sys.argv[0]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if launched and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.workload in ("c3", "fe") and world > 1:
        raise SystemExit(f"{args.workload} runs on one GPU (c3 is a sequential replay, SURVEY 8e); use --gpus 1")
    if args.workload == "c3":
        return run_c3(args, WORKLOADS["c3"]) or 0
    if args.workload == "fe":
        return run_fe(args, WORKLOADS["fe"]) or 0
    dd = Dist()
    if args.workload == "c4":
        return run_c4(args, WORKLOADS["c4"], dd, c4_backend)
    return run_replicas(args, WORKLOADS[args.workload], dd)


if __name__ == "__main__":
    sys.exit(main())
