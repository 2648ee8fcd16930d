"""Seeded synthetic LiDAR sequences (SURVEY.md §8(d) "Synthetic scan generator").

The reference's dataset (SUSCape CARLA npz: pos1, pos2, gt, s_fg_mask, ...) is not in the
repository and there is no network, so scans are ray-cast here:

* elevations at the bin centres of the reference's ring mapping (src/frameFeature.cpp:57-71):
  64 rows -> 2 - k/3 (k = 0..32) and -8.83 - m/2 (m = 1..31); 16 rows -> -15 + 2k.  A
  float32/float64 atan difference can therefore never move a point across a row edge;
* azimuth-major emission order (all beams per azimuth step, like a spinning sensor) -- or, with
  layout="carla", the layout of the reference's own data (launch/run_noSeg.launch:4 reads a
  road-removed CARLA set, .../rm_road/SF/04): channel-major order as CARLA's ray-cast LiDAR stores
  a sweep (every point of channel 0 in azimuth order, then channel 1, ...), no point for a ray
  without a return within the 100 m range (CARLA drops those; Scenario_Traj.py:307-315 leaves its
  drop-off on), no road points (ground returns with |y| < ROAD_HALF in the world, rm_road; the
  sidewalks and the ground off the street stay), and a uniform random drop-off down to
  exactly n_rows * n_az points per frame (oversample x as many rays are cast), so every frame
  has the bench's size but ragged rows;
* world: ground plane z = -2.5, a street of box buildings, poles (vertical cylinders), a
  100 m "sky dome" for rays that hit nothing, and moving cars (dynamic points, ~8 %);
* ego motion ~1 m/frame with a bounded heading (ego_yaw); range noise sigma 0.01 m plus 1e-4 m jitter so
  k-NN distances are tie-free;
* flow = pos1 expressed in frame k+1 coordinates minus pos1 (Generate_Sceneflow.py
  semantics); dynamic points include their object's motion.  s_fg_mask = 1 on movers.

Everything is computed in float64 with torch (CPU or GPU) and returned as float32.
"""
from __future__ import annotations

import math

import torch

SEED_BASE = 20240000


def elevations_deg(n_rows: int) -> torch.Tensor:
    if n_rows == 64:
        e = [2.0 - k / 3.0 for k in range(33)] + [-8.83 - m / 2.0 for m in range(1, 32)]
    elif n_rows == 16:
        e = [-15.0 + 2.0 * k for k in range(16)]
    else:
        raise ValueError("n_rows must be 16 or 64")
    return torch.tensor(e, dtype=torch.float64)


def _gen(seed: int) -> torch.Generator:
    g = torch.Generator()
    g.manual_seed(seed)
    return g


class Scene:
    """A static street world plus moving cars, deterministic in `seq`."""

    def __init__(self, seq: int = 0, n_buildings: int = 48, n_poles: int = 40, n_cars: int = 6):
        g = _gen(SEED_BASE + seq * 10000 + 9999)
        u = lambda *s: torch.rand(*s, generator=g, dtype=torch.float64)
        boxes = []
        for side in (-1.0, 1.0):
            x = -60.0
            for _ in range(n_buildings // 2):
                length = 8.0 + 14.0 * float(u(1))
                gap = 1.0 + 5.0 * float(u(1))
                depth = 6.0 + 10.0 * float(u(1))
                y0 = side * (9.0 + 4.0 * float(u(1)))
                h = 4.0 + 16.0 * float(u(1))
                ylo, yhi = (y0, y0 + side * depth) if side > 0 else (y0 - depth, y0)
                ylo, yhi = min(ylo, yhi), max(ylo, yhi)
                boxes.append([x, ylo, -2.5, x + length, yhi, -2.5 + h])
                x += length + gap
        self.boxes = torch.tensor(boxes, dtype=torch.float64)
        px = -50.0 + torch.arange(n_poles, dtype=torch.float64) * 16.0 + 3.0 * u(n_poles)
        py = torch.where(torch.arange(n_poles) % 2 == 0, torch.tensor(6.5), torch.tensor(-6.5))
        py = py.to(torch.float64) + 0.3 * u(n_poles)
        self.poles = torch.stack([px, py, 0.15 + 0.1 * u(n_poles), torch.full((n_poles,), 3.5)], 1)
        cars = []
        for c in range(n_cars):
            # lanes clear of the ego path (|y| <~ 2 m, ego_yaw) and of the poles (|y| ~ 6.5)
            lane = [-3.5, 3.5, -5.0, 5.0][c % 4]
            x0 = 5.0 + 25.0 * c + 10.0 * float(u(1))
            vx = (1.6 + 0.8 * float(u(1))) * (1.0 if lane > 0 else -1.0)
            cars.append([x0, lane, vx, 0.05 * (float(u(1)) - 0.5)])
        self.cars = torch.tensor(cars, dtype=torch.float64)  # x0, y, vx, vy
        self.car_half = torch.tensor([2.3, 0.95, 0.75], dtype=torch.float64)

    # Cars stay in a window around the ego (x relative to frame * EGO_SPEED in [CAR_LO, CAR_LO +
    # CAR_SPAN), wrapping round): a car that leaves it ahead or behind re-enters at the other end,
    # so the dynamic-point share stays steady along a sequence of any length, as in the CARLA
    # sequences the reference replays (before round 6 the cars drifted out of range: ~2 % dynamic
    # points at the first frames, none after frame ~60).  The motion within a frame (the flow's
    # velocity) is unchanged.
    CAR_LO, CAR_SPAN = -30.0, 70.0

    def car_boxes(self, frame: int) -> torch.Tensor:
        c = self.cars
        ego = frame * EGO_SPEED
        cx = ego + self.CAR_LO + torch.remainder(c[:, 0] + frame * c[:, 2] - ego - self.CAR_LO, self.CAR_SPAN)
        cy = c[:, 1] + frame * c[:, 3]
        cz = torch.full_like(cx, -2.5 + self.car_half[2].item())
        lo = torch.stack([cx, cy, cz], 1) - self.car_half
        hi = torch.stack([cx, cy, cz], 1) + self.car_half
        return torch.cat([lo, hi], 1)


EGO_SPEED = 1.0           # m per frame (ego_pose / ego_poses default speed)


def ego_yaw(seq: int, frame: int, yaw_rate: float = 0.004) -> float:
    """Heading of frame k: yaw0 + yaw_rate k for the first 15 frames, then a triangle wave of the
    same slope between +/- c0 (c0 = the heading reached at frame 15), whose mean is zero, so the
    lateral offset stays within ~2 m of the street axis however long the sequence (a constant
    yaw rate drove long sequences into the buildings, |y| > 9 m, after ~70 frames)."""
    yaw0 = 0.002 * ((seq * 7919) % 11 - 5)
    if frame <= 15:
        return yaw0 + yaw_rate * frame
    c0 = yaw0 + 15 * yaw_rate
    half = 2.0 * c0 / yaw_rate                      # frames from +c0 down to -c0
    u = math.fmod(frame - 15, 2.0 * half)
    return c0 - yaw_rate * u if u <= half else -c0 + yaw_rate * (u - half)


def ego_pose(seq: int, frame: int, speed: float = 1.0, yaw_rate: float = 0.004):
    """Sensor pose in the world: (R [3,3], p [3]) float64.  Constant speed, bounded heading."""
    p = torch.zeros(3, dtype=torch.float64)
    for k in range(frame):
        yk = ego_yaw(seq, k, yaw_rate)
        p = p + speed * torch.tensor([math.cos(yk), math.sin(yk), 0.0], dtype=torch.float64)
    y = ego_yaw(seq, frame, yaw_rate)
    c, s = math.cos(y), math.sin(y)
    R = torch.tensor([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]], dtype=torch.float64)
    return R, p


def _ray_boxes(o, d, boxes):
    """slab test: rays (o [3], d [n,3]) vs AABBs [b,6] -> t [n] (inf if no hit) and box id."""
    inv = 1.0 / torch.where(d.abs() < 1e-12, torch.full_like(d, 1e-12), d)
    lo = (boxes[None, :, 0:3] - o) * inv[:, None, :]
    hi = (boxes[None, :, 3:6] - o) * inv[:, None, :]
    tmin = torch.minimum(lo, hi).amax(2)
    tmax = torch.maximum(lo, hi).amin(2)
    hit = (tmax >= tmin) & (tmax > 0.5)
    t = torch.where(hit, torch.where(tmin > 0.5, tmin, tmax), torch.full_like(tmin, math.inf))
    tb, ib = t.min(1)
    return tb, ib


def _ray_poles(o, d, poles):
    dx, dy = d[:, 0:1], d[:, 1:2]
    ox = o[0] - poles[None, :, 0]
    oy = o[1] - poles[None, :, 1]
    a = dx * dx + dy * dy
    b = 2.0 * (ox * dx + oy * dy)
    c = ox * ox + oy * oy - poles[None, :, 2] ** 2
    disc = b * b - 4 * a * c
    sq = torch.sqrt(torch.clamp(disc, min=0.0))
    t = (-b - sq) / (2 * a)
    z = o[2] + t * d[:, 2:3]
    ok = (disc > 0) & (t > 0.5) & (z > -2.5) & (z < -2.5 + poles[None, :, 3])
    t = torch.where(ok, t, torch.full_like(t, math.inf))
    return t.min(1).values


LAYOUTS = ("azimuth", "carla")
ROAD_HALF = 6.0           # the road: |y| < 6 m in the world (poles stand at 6.5, buildings from 9)
CARLA_OVERSAMPLE = 3      # rays cast per kept point in the "carla" layout (ample: ~40 % return)


def scan(seq: int, frame: int, n_rows: int = 64, n_az: int = 1875, device="cpu",
         scene: Scene | None = None, layout: str = "azimuth"):
    """One synthetic frame -> dict(pos1 [N,3] f32, flow [N,3] f32, s_fg_mask [N] u8).

    N = n_rows * n_az exactly.  layout "azimuth": every ray returns (rays that hit nothing land on
    a 100 m dome), azimuth-major.  layout "carla": CARLA_OVERSAMPLE x n_az rays per channel,
    channel-major; rays without an object return (dome or road) are dropped, then a uniform
    random drop-off keeps exactly N points in their order (module docstring)."""
    if layout not in LAYOUTS:
        raise ValueError(f"layout must be one of {LAYOUTS}")
    scene = scene or Scene(seq)
    g = _gen(SEED_BASE + seq * 10000 + frame)
    carla = layout == "carla"
    n_keep = n_rows * n_az
    if carla:
        n_az = CARLA_OVERSAMPLE * n_az
    el = elevations_deg(n_rows) * (math.pi / 180.0)
    az0 = 2 * math.pi * torch.rand(1, generator=g, dtype=torch.float64).item() / n_az
    az = az0 + 2 * math.pi * torch.arange(n_az, dtype=torch.float64) / n_az
    ce, se = torch.cos(el), torch.sin(el)
    # azimuth-major: index = a * n_rows + r
    ds = torch.stack([ce[None, :] * torch.cos(az)[:, None], ce[None, :] * torch.sin(az)[:, None],
                      se[None, :].expand(n_az, n_rows)], 2).reshape(-1, 3)
    if carla:                                   # channel-major: index = r * n_az + a
        ds = ds.view(n_az, n_rows, 3).transpose(0, 1).reshape(-1, 3).contiguous()
    noise_r = 0.01 * torch.randn(ds.shape[0], generator=g, dtype=torch.float64)
    jitter = 1e-4 * (torch.rand(ds.shape[0], 3, generator=g, dtype=torch.float64) - 0.5)
    ds = ds.to(device)
    R, p = ego_pose(seq, frame)
    R, p = R.to(device), p.to(device)
    dw = ds @ R.T
    n = dw.shape[0]
    t = torch.full((n,), 100.0, dtype=torch.float64, device=device)
    mover = torch.full((n,), -1, dtype=torch.long, device=device)
    obj = torch.zeros(n, dtype=torch.bool, device=device)      # returned from an object
    tg = torch.where(dw[:, 2] < -1e-9, (-2.5 - p[2]) / dw[:, 2], torch.full_like(t, math.inf))
    t = torch.minimum(t, tg)
    chunk = 1 << 16
    boxes = scene.boxes.to(device)
    cars = scene.car_boxes(frame).to(device)
    poles = scene.poles.to(device)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        tb, _ = _ray_boxes(p, dw[s:e], boxes)
        tp = _ray_poles(p, dw[s:e], poles)
        tc, ic = _ray_boxes(p, dw[s:e], cars)
        to = torch.minimum(tb, tp)
        ts = torch.minimum(t[s:e], to)
        car_hit = tc < ts
        # a return that is kept: an object, or ground off the road (|y| >= ROAD_HALF: sidewalks,
        # the ground between and behind the buildings); road points are removed (rm_road)
        ground = ~car_hit & ~(to < t[s:e]) & (t[s:e] < 100.0)
        yw = p[1] + t[s:e] * dw[s:e, 1]
        obj[s:e] = car_hit | (to < t[s:e]) | (ground & (yw.abs() >= ROAD_HALF))
        t[s:e] = torch.where(car_hit, tc, ts)
        mover[s:e] = torch.where(car_hit, ic, torch.full_like(ic, -1))
    t = torch.clamp(t, max=100.0) + noise_r.to(device)
    pos1 = ds * t[:, None] + jitter.to(device)
    # flow: same physical point in frame k+1 coordinates (movers displaced by their velocity)
    W = pos1 @ R.T + p
    vel = torch.zeros_like(W)
    car_v = torch.cat([scene.cars[:, 2:4], torch.zeros(scene.cars.shape[0], 1, dtype=torch.float64)], 1).to(device)
    m = mover >= 0
    vel[m] = car_v[mover[m]]
    R2, p2 = ego_pose(seq, frame + 1)
    R2, p2 = R2.to(device), p2.to(device)
    pos2 = (W + vel - p2) @ R2
    pos1f = pos1.to(torch.float32)
    flow = (pos2 - pos1f.to(torch.float64)).to(torch.float32)
    out = dict(pos1=pos1f, flow=flow, s_fg_mask=m.to(torch.uint8))
    if carla:
        keep = carla_keep(obj.cpu(), n_keep, torch.rand(n, generator=g, dtype=torch.float64))
        out = {k: v[keep.to(v.device)] for k, v in out.items()}
    return out


def carla_keep(returned: torch.Tensor, n_keep: int, u: torch.Tensor) -> torch.Tensor:
    """The random drop-off of the "carla" layout: of the rays that returned (bool [n]), the
    n_keep with the smallest keys u (uniform, [n]) -> a bool mask that keeps their order."""
    key = torch.where(returned, u, torch.full_like(u, 2.0))
    if int(returned.sum()) < n_keep:
        raise ValueError(f"carla layout: {int(returned.sum())} returns for {n_keep} points "
                         f"(raise CARLA_OVERSAMPLE)")
    thr = torch.kthvalue(key, n_keep).values
    keep = key <= thr
    assert int(keep.sum()) == n_keep
    return keep


_SYNTH_LIB = None


def _synth_lib():
    """libssf_synth.so (csrc/synth.hip): the batched GPU form of scan(), for bench data."""
    global _SYNTH_LIB
    if _SYNTH_LIB is None:
        import ctypes as C
        import os
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libssf_synth.so")
        lib = C.CDLL(path)
        lib.ssf_synth_scan_batch.restype = C.c_int
        lib.ssf_synth_scan_batch.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                             C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                             C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]
        _SYNTH_LIB = lib
    return _SYNTH_LIB


def ego_poses(seq: int, n_frames: int, speed: float = 1.0, yaw_rate: float = 0.004):
    """ego_pose(seq, k) for k < n_frames at once -> (R [n,3,3], p [n,3]) numpy float64."""
    import numpy as np
    y = np.array([ego_yaw(seq, k, yaw_rate) for k in range(n_frames)], dtype=np.float64)
    step = speed * np.stack([np.cos(y), np.sin(y), np.zeros_like(y)], 1)
    p = np.concatenate([np.zeros((1, 3)), np.cumsum(step, 0)[:-1]], 0)
    c, s = np.cos(y), np.sin(y)
    R = np.zeros((n_frames, 3, 3))
    R[:, 0, 0], R[:, 0, 1], R[:, 1, 0], R[:, 1, 1], R[:, 2, 2] = c, -s, s, c, 1.0
    return R, p


class BatchScanner:
    """scan() for S sequences at once on the GPU (libssf_synth.so): the same scenes, sensor and
    ego motion as scan(), one ray per thread; the range noise and the jitter come from a
    counter-based hash instead of torch's CPU generator.  Bench / test data only."""

    def __init__(self, seqs, n_frames: int, n_rows: int = 64, n_az: int = 1875, device="cuda",
                 layout: str = "azimuth", start=None):
        """start: optional first frame per sequence (frame(k) gives frame start[j] + k of sequence
        j), so a batch's sequences sit at different points of their trajectories."""
        import numpy as np
        if layout not in LAYOUTS:
            raise ValueError(f"layout must be one of {LAYOUTS}")
        self.layout = layout
        self.seqs, self.n_rows, self.n_az, self.device = list(seqs), n_rows, n_az, torch.device(device)
        self.start = [0] * len(self.seqs) if start is None else [int(v) for v in start]
        if len(self.start) != len(self.seqs) or min(self.start, default=0) < 0:
            raise ValueError("start must hold one frame index >= 0 per sequence")
        self.scenes = [Scene(s) for s in self.seqs]
        self.poses = [ego_poses(s, n_frames + st + 1) for s, st in zip(self.seqs, self.start)]
        sc = self.scenes[0]
        self.n_box, self.n_pole, self.n_car = sc.boxes.shape[0], sc.poles.shape[0], sc.cars.shape[0]
        self.rec = 25 + 6 * self.n_box + 4 * self.n_pole + 9 * self.n_car
        self.elev = (elevations_deg(n_rows) * (math.pi / 180.0)).to(self.device)
        self._np = np

    def frame(self, k0: int, pos: torch.Tensor, flow: torch.Tensor):
        """frame start[j] + k0 of every sequence j into pos / flow [S * N, 3] f32 (device,
        contiguous)."""
        import ctypes as C
        np = self._np
        S, N = len(self.seqs), self.n_rows * self.n_az
        assert pos.shape == (S * N, 3) and flow.shape == (S * N, 3) and pos.is_contiguous() and flow.is_contiguous()
        carla = self.layout == "carla"
        n_az = CARLA_OVERSAMPLE * self.n_az if carla else self.n_az
        if carla:                                   # every ray first, then the drop-off to N
            M = self.n_rows * n_az
            rpos = torch.empty((S * M, 3), dtype=torch.float32, device=self.device)
            rflow = torch.empty_like(rpos)
            rkey = torch.empty(S * M, dtype=torch.float64, device=self.device)
        else:
            rpos, rflow, rkey = pos, flow, None
        prm = np.zeros((S, self.rec))
        seeds = np.zeros(S, dtype=np.uint64)
        for j, (seq, sc) in enumerate(zip(self.seqs, self.scenes)):
            k = k0 + self.start[j]
            R, p = self.poses[j]
            az0 = 2 * math.pi * torch.rand(1, generator=_gen(SEED_BASE + seq * 10000 + k),
                                           dtype=torch.float64).item() / n_az
            car = sc.car_boxes(k).numpy()
            carv = np.concatenate([sc.cars[:, 2:4].numpy(), np.zeros((self.n_car, 1))], 1)
            prm[j] = np.concatenate([R[k].ravel(), p[k], R[k + 1].ravel(), p[k + 1], [az0],
                                     sc.boxes.numpy().ravel(), sc.poles.numpy().ravel(), car.ravel(),
                                     carv.ravel()])
            seeds[j] = (SEED_BASE + seq * 10000 + k) * 0x9E3779B97F4A7C15 % (1 << 64)
        d_prm = torch.from_numpy(prm).to(self.device)
        d_seeds = torch.from_numpy(seeds.view(np.int64)).to(self.device)
        st = torch.cuda.current_stream(self.device).cuda_stream
        rc = _synth_lib().ssf_synth_scan_batch(
            C.c_void_p(st), S, self.n_rows, n_az, C.c_void_p(self.elev.data_ptr()),
            C.c_void_p(d_prm.data_ptr()), self.rec, self.n_box, self.n_pole, self.n_car,
            C.c_void_p(d_seeds.data_ptr()), 1 if carla else 0, C.c_void_p(rpos.data_ptr()),
            C.c_void_p(rflow.data_ptr()), None if rkey is None else C.c_void_p(rkey.data_ptr()))
        if rc != 0:
            raise RuntimeError(f"ssf_synth_scan_batch failed: hipError {rc}")
        d_prm.record_stream(torch.cuda.current_stream(self.device))
        d_seeds.record_stream(torch.cuda.current_stream(self.device))
        if carla:                                   # per sequence the N smallest keys, in order
            kv = rkey.view(S, -1)
            if int((kv < 2.0).sum(1).min()) < N:
                raise ValueError("carla layout: too few returns for the frame size (raise CARLA_OVERSAMPLE)")
            thr = torch.kthvalue(kv, N, dim=1).values
            keep = (kv <= thr[:, None]).view(-1)
            sel = torch.nonzero(keep).view(-1)
            if sel.numel() != S * N:
                raise RuntimeError("carla layout: tied selection keys")
            torch.index_select(rpos, 0, sel, out=pos)
            torch.index_select(rflow, 0, sel, out=flow)


def relative_pose(seq: int, frame_last: int, frame_curr: int):
    """Ground-truth T_last<-curr as (q_xyzw, t) float64 tuples (lidarOdometry q_last_curr)."""
    Rl, pl = ego_pose(seq, frame_last)
    Rc, pc = ego_pose(seq, frame_curr)
    R = Rl.T @ Rc
    t = Rl.T @ (pc - pl)
    w = math.sqrt(max(0.0, 1.0 + R[0, 0] + R[1, 1] + R[2, 2])) / 2.0
    q = (float((R[2, 1] - R[1, 2]) / (4 * w)), float((R[0, 2] - R[2, 0]) / (4 * w)),
         float((R[1, 0] - R[0, 1]) / (4 * w)), w)
    return q, tuple(float(v) for v in t)
