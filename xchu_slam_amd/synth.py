"""Deterministic synthetic LiDAR world for the NDT benchmark / parity workloads.

No KITTI scans exist in the container or on the GPU box, so the BASELINE configs are restated on a seeded
synthetic world W: an undulating ground plane (z = 0.2 sin(x/15) cos(y/11)), box buildings (vertical facades)
and poles.  The target ("localmap") samples every surface of W inside a square map; the source ("scan") is a
LiDAR-like sample of the surfaces around a sensor pose (density ~ 1/r, range 1..max_range m), expressed in
the sensor frame.  The true sensor pose is known, so alignment accuracy is checkable.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np


@dataclass
class World:
    half: float                 # map half-size (m)
    buildings: np.ndarray       # (B, 6): cx, cy, w, d, h, yaw
    poles: np.ndarray           # (P, 4): x, y, r, h
    noise: float = 0.02

    # ----------------------------------------------------------------- surfaces
    def _ground(self, rng, n, cx=0.0, cy=0.0, R=None):
        if R is None:
            x = rng.uniform(-self.half, self.half, n)
            y = rng.uniform(-self.half, self.half, n)
        else:
            rr = R * np.sqrt(rng.uniform(0.0, 1.0, n))
            th = rng.uniform(0.0, 2 * math.pi, n)
            x = cx + rr * np.cos(th)
            y = cy + rr * np.sin(th)
        z = 0.2 * np.sin(x / 15.0) * np.cos(y / 11.0)
        return np.stack([x, y, z], 1)

    def _walls(self, rng, n, sel=None):
        b = self.buildings if sel is None else self.buildings[sel]
        if len(b) == 0 or n == 0:
            return np.zeros((0, 3))
        area = 2 * (b[:, 2] + b[:, 3]) * b[:, 4]
        k = rng.choice(len(b), size=n, p=area / area.sum())
        cx, cy, w, d, h, yaw = (b[k, i] for i in range(6))
        per = 2 * (w + d)
        s = rng.uniform(0, 1, n) * per
        u = np.where(s < w, s - w / 2, np.where(s < w + d, w / 2, np.where(s < 2 * w + d, w / 2 - (s - w - d), -w / 2)))
        v = np.where(s < w, -d / 2, np.where(s < w + d, -d / 2 + (s - w), np.where(s < 2 * w + d, d / 2, d / 2 - (s - 2 * w - d))))
        z = rng.uniform(0, 1, n) * h
        c, sn = np.cos(yaw), np.sin(yaw)
        return np.stack([cx + c * u - sn * v, cy + sn * u + c * v, z], 1)

    def _poles(self, rng, n, sel=None):
        p = self.poles if sel is None else self.poles[sel]
        if len(p) == 0 or n == 0:
            return np.zeros((0, 3))
        k = rng.integers(0, len(p), n)
        th = rng.uniform(0, 2 * math.pi, n)
        z = rng.uniform(0, 1, n) * p[k, 3]
        return np.stack([p[k, 0] + p[k, 2] * np.cos(th), p[k, 1] + p[k, 2] * np.sin(th), z], 1)

    def surface_areas(self):
        ground = (2 * self.half) ** 2
        walls = float(np.sum(2 * (self.buildings[:, 2] + self.buildings[:, 3]) * self.buildings[:, 4])) if len(self.buildings) else 0.0
        poles = float(np.sum(2 * math.pi * self.poles[:, 2] * self.poles[:, 3])) if len(self.poles) else 0.0
        return ground, walls, poles

    # ----------------------------------------------------------------- clouds
    def target(self, density: float, seed: int) -> np.ndarray:
        """Localmap sample of all surfaces at `density` points/m^2, world frame, (M, 3) float32.

        The ground is stratified per 1 m^2 cell (every cell receives round(density) points) so that voxel
        occupancy is even, as in a keyframe-merged, 1 m-downsampled localmap; facades and poles are sampled
        uniformly by area."""
        rng = np.random.default_rng(seed)
        k = int(round(density))
        n_cells = int(2 * self.half)
        ii, jj = np.meshgrid(np.arange(n_cells), np.arange(n_cells), indexing="ij")
        base = np.stack([ii.ravel(), jj.ravel()], 1).astype(np.float64) - self.half
        gxy = np.repeat(base, k, axis=0) + rng.uniform(0.0, 1.0, (base.shape[0] * k, 2))
        gz = 0.2 * np.sin(gxy[:, 0] / 15.0) * np.cos(gxy[:, 1] / 11.0)
        ground = np.concatenate([gxy, gz[:, None]], 1)
        _, aw, ap = self.surface_areas()
        walls = self._walls(rng, int(density * aw))
        poles = self._poles(rng, int(density * ap))
        pts = np.concatenate([ground, walls, poles])
        pts += rng.normal(0, self.noise, pts.shape)
        return pts[rng.permutation(len(pts))].astype(np.float32)

    def scan(self, n_points: int, center_xy, seed: int, max_range: float = 60.0) -> np.ndarray:
        """LiDAR-like sample around (cx, cy) in the world frame: density ~ 1/r up to max_range."""
        rng = np.random.default_rng(seed)
        cx, cy = float(center_xy[0]), float(center_xy[1])
        out = []
        need = n_points
        while need > 0:
            m = int(need * 1.6) + 64
            # ground with density ~ 1/r: r uniform in [1, R]
            rr = rng.uniform(1.0, max_range, m)
            th = rng.uniform(0, 2 * math.pi, m)
            g = np.stack([cx + rr * np.cos(th), cy + rr * np.sin(th)], 1)
            gz = 0.2 * np.sin(g[:, 0] / 15.0) * np.cos(g[:, 1] / 11.0)
            ground = np.concatenate([g, gz[:, None]], 1)
            # structures near the sensor
            bd = np.hypot(self.buildings[:, 0] - cx, self.buildings[:, 1] - cy) if len(self.buildings) else np.zeros(0)
            sel_b = np.nonzero(bd < max_range + 20)[0]
            pd = np.hypot(self.poles[:, 0] - cx, self.poles[:, 1] - cy) if len(self.poles) else np.zeros(0)
            sel_p = np.nonzero(pd < max_range)[0]
            walls = self._walls(rng, m, sel_b) if len(sel_b) else np.zeros((0, 3))
            poles = self._poles(rng, m // 8, sel_p) if len(sel_p) else np.zeros((0, 3))
            cand = np.concatenate([ground[: int(0.55 * m)], walls[: int(0.4 * m)], poles])
            r = np.hypot(cand[:, 0] - cx, cand[:, 1] - cy)
            keep = (r > 1.0) & (r < max_range) & (np.abs(cand[:, 0]) < self.half) & (np.abs(cand[:, 1]) < self.half)
            # thin far structure points (density ~ 1/r for walls too)
            keep &= rng.uniform(0, 1, len(cand)) < np.minimum(1.0, 15.0 / np.maximum(r, 1.0))
            cand = cand[keep]
            out.append(cand)
            need -= len(cand)
        pts = np.concatenate(out)[rng.permutation(sum(len(o) for o in out))[:n_points]]
        pts += rng.normal(0, self.noise, pts.shape)
        return pts.astype(np.float32)


def make_world(seed: int = 0, half: float = 210.0, n_buildings: int | None = None, n_poles: int | None = None) -> World:
    rng = np.random.default_rng(seed)
    area = (2 * half) ** 2
    nb = n_buildings if n_buildings is not None else int(area / 2500)
    npl = n_poles if n_poles is not None else int(area / 900)
    b = np.stack([rng.uniform(-half + 20, half - 20, nb), rng.uniform(-half + 20, half - 20, nb), rng.uniform(8, 30, nb),
                  rng.uniform(8, 30, nb), rng.uniform(4, 18, nb), rng.uniform(0, math.pi, nb)], 1) if nb else np.zeros((0, 6))
    p = np.stack([rng.uniform(-half + 5, half - 5, npl), rng.uniform(-half + 5, half - 5, npl), np.full(npl, 0.15),
                  rng.uniform(4, 8, npl)], 1) if npl else np.zeros((0, 4))
    return World(half=half, buildings=b, poles=p)


def pose_matrix(x, y, z, roll, pitch, yaw) -> np.ndarray:
    """Pose6D2Matrix (common.h:64-71): T(x,y,z) * Rz(yaw) * Ry(pitch) * Rx(roll), float64."""
    cr, sr, cp, sp, cy, sy = math.cos(roll), math.sin(roll), math.cos(pitch), math.sin(pitch), math.cos(yaw), math.sin(yaw)
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    T = np.eye(4)
    T[:3, :3] = Rz @ Ry @ Rx
    T[:3, 3] = [x, y, z]
    return T


@dataclass
class Pair:
    target: np.ndarray      # (M, 3) world frame
    source: np.ndarray      # (N, 3) sensor frame
    true_pose: np.ndarray   # 4x4 sensor -> world
    guess: np.ndarray       # 4x4 perturbed


def make_pair(world: World, density: float, n_source: int, seed: int, max_range: float = 60.0,
              perturb=(0.3, 0.3, 0.05, 0.5, 0.5, 1.0)) -> Pair:
    """One scan->localmap pair: guess = true pose perturbed by (m, m, m, deg, deg, deg)."""
    rng = np.random.default_rng(seed)
    lim = max(world.half - max_range - 5.0, 0.0)
    cx, cy = rng.uniform(-lim, lim, 2) if lim > 0 else (0.0, 0.0)
    yaw = rng.uniform(-math.pi, math.pi)
    true = pose_matrix(cx, cy, 1.73, rng.normal(0, 0.01), rng.normal(0, 0.01), yaw)
    tgt = world.target(density, seed + 1000)
    scan_w = world.scan(n_source, (cx, cy), seed + 5000, max_range)
    inv = np.linalg.inv(true)
    src = (scan_w.astype(np.float64) @ inv[:3, :3].T + inv[:3, 3]).astype(np.float32)
    sgn = rng.choice([-1.0, 1.0], 6)
    d = [perturb[0] * sgn[0], perturb[1] * sgn[1], perturb[2] * sgn[2], math.radians(perturb[3]) * sgn[3],
         math.radians(perturb[4]) * sgn[4], math.radians(perturb[5]) * sgn[5]]
    guess = true @ pose_matrix(*d)
    return Pair(target=tgt, source=src, true_pose=true, guess=guess)


def to_xyz4(p: np.ndarray) -> np.ndarray:
    out = np.ones((p.shape[0], 4), np.float32)
    out[:, :3] = p
    return out


# ----------------------------------------------------------------- C3 replay sequences
_CAM_TO_WORLD = np.array([[0.0, 0.0, 1.0], [-1.0, 0.0, 0.0], [0.0, -1.0, 0.0]])  # KITTI camera (x right, y down, z fwd) -> z-up


def kitti_poses(tum: np.ndarray, start: int = 0, count: int | None = None, stride: int = 1, height: float = 1.73) -> np.ndarray:
    """Sensor poses (K, 4, 4) in a z-up world from KITTI TUM ground truth (t tx ty tz qx qy qz qw, camera frame):
    axes remapped to x forward / y left / z up, the path centred on the origin, the sensor held at `height` above
    the flat synthetic ground (KITTI's ~25 m of elevation change is dropped; roll / pitch / yaw are kept)."""
    sel = tum[start:None if count is None else start + count * stride:stride]
    out = np.zeros((len(sel), 4, 4))
    centre = _CAM_TO_WORLD @ np.array([(tum[:, 1].min() + tum[:, 1].max()) / 2, 0.0, (tum[:, 3].min() + tum[:, 3].max()) / 2])
    for k, r in enumerate(sel):
        qx, qy, qz, qw = r[4:8]
        R = np.array([[1 - 2 * (qy * qy + qz * qz), 2 * (qx * qy - qz * qw), 2 * (qx * qz + qy * qw)],
                      [2 * (qx * qy + qz * qw), 1 - 2 * (qx * qx + qz * qz), 2 * (qy * qz - qx * qw)],
                      [2 * (qx * qz - qy * qw), 2 * (qy * qz + qx * qw), 1 - 2 * (qx * qx + qy * qy)]])
        out[k, :3, :3] = _CAM_TO_WORLD @ R @ _CAM_TO_WORLD.T
        t = _CAM_TO_WORLD @ r[1:4] - centre
        out[k, :3, 3] = [t[0], t[1], height]
        out[k, 3, 3] = 1.0
    return out


def make_world_for_path(seed: int, path_xy: np.ndarray, half: float, clearance: float = 12.0) -> World:
    """make_world with the buildings and poles that would stand on the driven path removed."""
    w = make_world(seed, half=half)
    if len(path_xy) == 0:
        return w

    def far(xy, r):
        d2 = ((xy[:, None, :] - path_xy[None, ::5, :]) ** 2).sum(-1)
        return d2.min(1) > r * r

    if len(w.buildings):
        rad = 0.5 * np.hypot(w.buildings[:, 2], w.buildings[:, 3])
        keep = np.array([far(w.buildings[i:i + 1, :2], rad[i] + clearance)[0] for i in range(len(w.buildings))])
        w.buildings = w.buildings[keep]
    if len(w.poles):
        w.poles = w.poles[far(w.poles[:, :2], clearance / 3)]
    return w


def make_street_world(seed: int, path_xy: np.ndarray, half: float, spacing: float = 20.0, setback: float = 9.0) -> World:
    """make_world_for_path plus street furniture along the driven path: facades set back `setback`..+8 m on both
    sides (75 % of `spacing` slots, aligned with the road) and poles 4-6 m from the centre line, so that every
    stretch of the replay sees vertical structure (a KITTI-like residential street, not an open field)."""
    w = make_world_for_path(seed, path_xy, half)
    if len(path_xy) < 2:
        return w
    rng = np.random.default_rng(seed + 77)
    seg = np.hypot(*np.diff(path_xy, axis=0).T)
    arc = np.concatenate([[0.0], np.cumsum(seg)])
    blds, poles = [], []
    for m in np.arange(0.0, arc[-1], spacing):
        i = min(int(np.searchsorted(arc, m)), len(path_xy) - 1)
        j0, j1 = max(0, i - 5), min(len(path_xy) - 1, i + 5)
        t = path_xy[j1] - path_xy[j0]
        if np.hypot(*t) < 1e-6:
            continue
        t = t / np.hypot(*t)
        nrm = np.array([-t[1], t[0]])
        yaw = math.atan2(t[1], t[0])
        for side in (-1.0, 1.0):
            if rng.random() < 0.75:
                wd, dp = rng.uniform(8.0, 18.0), rng.uniform(8.0, 16.0)
                c = path_xy[i] + side * (rng.uniform(setback, setback + 8.0) + dp / 2) * nrm + rng.uniform(-3, 3) * t
                blds.append([c[0], c[1], wd, dp, rng.uniform(5.0, 15.0), yaw])
            if rng.random() < 0.6:
                c = path_xy[i] + side * rng.uniform(4.0, 6.0) * nrm + rng.uniform(-spacing / 2, spacing / 2) * t
                poles.append([c[0], c[1], 0.15, rng.uniform(4.0, 8.0)])
    if blds:
        b = np.array(blds)
        # drop facades that a curve or a crossing street brings onto the road: nearest path point must clear the
        # building's half-diagonal plus 4 m
        rad = 0.5 * np.hypot(b[:, 2], b[:, 3])
        d2 = ((b[:, None, :2] - path_xy[None, ::2, :]) ** 2).sum(-1).min(1)
        b = b[np.sqrt(d2) > rad + 4.0]
        w.buildings = np.concatenate([w.buildings, b]) if len(w.buildings) else b
    if poles:
        pl = np.array(poles)
        d2 = ((pl[:, None, :2] - path_xy[None, ::2, :]) ** 2).sum(-1).min(1)
        pl = pl[np.sqrt(d2) > 3.0]
        w.poles = np.concatenate([w.poles, pl]) if len(w.poles) else pl
    return w


def sensor_scan(world: World, pose: np.ndarray, n_points: int, seed: int, max_range: float = 60.0) -> np.ndarray:
    """A LiDAR-like scan of `world` taken at `pose` (sensor -> world), returned in the sensor frame (N, 3) f32."""
    pts_w = world.scan(n_points, (pose[0, 3], pose[1, 3]), seed, max_range).astype(np.float64)
    inv = np.linalg.inv(pose)
    return (pts_w @ inv[:3, :3].T + inv[:3, 3]).astype(np.float32)


def make_sequence(tum: np.ndarray, n_scans: int, n_points: int, seed: int = 0, start: int = 0, max_range: float = 60.0):
    """C3 replay input: (world, sensor poses (K,4,4), scans [K x (N,3) f32 sensor frame])."""
    poses = kitti_poses(tum, start=start, count=n_scans)
    all_xy = kitti_poses(tum)[:, :2, 3]
    half = float(np.abs(all_xy).max()) + max_range + 30.0
    world = make_street_world(seed, all_xy, half)
    scans = [sensor_scan(world, poses[k], n_points, seed + 7919 * (k + 1), max_range) for k in range(len(poses))]
    return world, poses, scans


def write_sequence(path: str, poses: np.ndarray, scans, stamps=None) -> None:
    """Binary sequence file for the C++ replay driver: "NDTSEQ01", int64 K, then per scan: int64 N, f64 stamp,
    f64[16] ground-truth pose (row-major), f32[N*3] points (sensor frame)."""
    with open(path, "wb") as f:
        f.write(b"NDTSEQ01")
        f.write(np.int64(len(scans)).tobytes())
        for k, s in enumerate(scans):
            s = np.ascontiguousarray(s, np.float32)
            f.write(np.int64(len(s)).tobytes())
            f.write(np.float64(0.1 * k if stamps is None else stamps[k]).tobytes())
            f.write(np.ascontiguousarray(poses[k], np.float64).tobytes())
            f.write(s.tobytes())


# ----------------------------------------------------------------- C4 batched replay pairs, generated on device
C4_PERTURB = (0.3, 0.3, 0.05, 0.5, 0.5, 1.0)


@dataclass
class DevicePairSpec:
    """Host half of one C4 pair: the small world + pose (numpy), point counts and the generator descriptor fields.
    The points themselves are made on the device by libndt_synth.so (bench infrastructure, csrc/synth_pairs.hip)."""
    index: int
    world_floats: np.ndarray    # ndt_synth.h world layout
    fields: dict                # SynthPairDesc fields
    n_target: int
    n_source: int
    true_pose: np.ndarray       # 4x4 sensor -> world
    guess: np.ndarray           # 4x4 perturbed


def c4_pair_spec(i: int, half: float = 210.0, density: float = 8.0, n_source: int = 120_000, max_range: float = 60.0,
                 noise: float = 0.02) -> DevicePairSpec:
    """Pair i of the C4 set: world and localmap from seed 1000+i, scan pose and scan from seed 5000+i.
    Same world model as make_pair (ground stratified per 1 m cell at round(density) points, facades and poles by area);
    a pure function of i, so every rank / shard count sees the same pair."""
    w = make_world(1000 + i, half=half)
    rng = np.random.default_rng(5000 + i)
    lim = max(half - max_range - 5.0, 0.0)
    cx, cy = rng.uniform(-lim, lim, 2) if lim > 0 else (0.0, 0.0)
    yaw = rng.uniform(-math.pi, math.pi)
    true = pose_matrix(cx, cy, 1.73, rng.normal(0, 0.01), rng.normal(0, 0.01), yaw)
    sgn = rng.choice([-1.0, 1.0], 6)
    p = C4_PERTURB
    d = [p[0] * sgn[0], p[1] * sgn[1], p[2] * sgn[2], math.radians(p[3]) * sgn[3], math.radians(p[4]) * sgn[4],
         math.radians(p[5]) * sgn[5]]
    guess = true @ pose_matrix(*d)
    b, pl = w.buildings, w.poles
    nb, npl = len(b), len(pl)
    area = 2 * (b[:, 2] + b[:, 3]) * b[:, 4]

    def cdf(wt):
        c = np.cumsum(wt) / max(wt.sum(), 1e-30)
        nz = np.nonzero(wt > 0)[0]
        if len(nz):
            c[nz[-1]:] = 1.0
        return c

    near_b = np.hypot(b[:, 0] - cx, b[:, 1] - cy) < max_range + 20
    near_p = np.hypot(pl[:, 0] - cx, pl[:, 1] - cy) < max_range
    world = np.concatenate([b.reshape(-1), cdf(area), cdf(area * near_b), pl.reshape(-1), cdf(near_p.astype(np.float64))])
    _, aw, ap = w.surface_areas()
    cells = int(2 * half)
    k = int(round(density))
    n_ground, n_walls, n_poles = cells * cells * k, int(density * aw), int(density * ap)
    m = n_ground + n_walls + n_poles
    hb = 1
    while (1 << (2 * hb)) < m:
        hb += 1
    inv = np.linalg.inv(true)
    fields = dict(seed_target=1000 + i, seed_source=5000 + i, nb=nb, np=npl, nb_near=int(near_b.sum()), np_near=int(near_p.sum()),
                  cells_side=cells, per_cell=k, perm_half_bits=hb, n_ground=n_ground, n_walls=n_walls, n_poles=n_poles,
                  n_source=n_source, half=half, noise=noise, max_range=max_range, cx=float(cx), cy=float(cy),
                  world_to_sensor=inv[:3, :4].reshape(-1))
    return DevicePairSpec(index=i, world_floats=world.astype(np.float32), fields=fields, n_target=m, n_source=n_source,
                          true_pose=true, guess=guess)


class SynthPairDescC(__import__("ctypes").Structure):
    """ctypes mirror of SynthPairDesc (xchu_slam_amd/csrc/ndt_synth.h)."""
    import ctypes as _C
    _fields_ = [("seed_target", _C.c_ulonglong), ("seed_source", _C.c_ulonglong), ("device", _C.c_int), ("nb", _C.c_int),
                ("np", _C.c_int), ("nb_near", _C.c_int), ("np_near", _C.c_int), ("cells_side", _C.c_int), ("per_cell", _C.c_int),
                ("perm_half_bits", _C.c_int), ("n_ground", _C.c_longlong), ("n_walls", _C.c_longlong), ("n_poles", _C.c_longlong),
                ("n_source", _C.c_int), ("half", _C.c_float), ("noise", _C.c_float), ("max_range", _C.c_float), ("cx", _C.c_float),
                ("cy", _C.c_float), ("world_to_sensor", _C.c_double * 12)]
    del _C


_synth_lib = None


def _load_synth():
    global _synth_lib
    if _synth_lib is None:
        import ctypes as C
        import os
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libndt_synth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} not found: build with make -C xchu_slam_amd/csrc")
        lib = C.CDLL(path)
        lib.ndt_synth_world_floats.restype = C.c_int
        lib.ndt_synth_world_floats.argtypes = [C.c_int, C.c_int]
        lib.ndt_synth_pair_device.restype = C.c_int
        lib.ndt_synth_pair_device.argtypes = [C.POINTER(SynthPairDescC), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        _synth_lib = lib
    return _synth_lib


def generate_pair_device(spec: DevicePairSpec, device: int, d_world: int, d_target: int, d_source: int) -> None:
    """Fill device buffers d_target (spec.n_target float4) and d_source (spec.n_source float4) with C4 pair spec.index;
    d_world: device scratch of len(spec.world_floats) floats.  Synchronous."""
    import ctypes as C
    lib = _load_synth()
    d = SynthPairDescC()
    for k, v in spec.fields.items():
        if k == "world_to_sensor":
            for j in range(12):
                d.world_to_sensor[j] = float(v[j])
        else:
            setattr(d, k, v)
    d.device = device
    w = np.ascontiguousarray(spec.world_floats, np.float32)
    assert len(w) == lib.ndt_synth_world_floats(d.nb, d.np)
    rc = lib.ndt_synth_pair_device(C.byref(d), w.ctypes.data_as(C.c_void_p), C.c_void_p(d_world), C.c_void_p(d_target),
                                   C.c_void_p(d_source))
    if rc != 0:
        raise RuntimeError(f"ndt_synth_pair_device failed ({rc})")
