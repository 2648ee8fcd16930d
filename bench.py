"""Benchmark: LiDAR front-end frames/sec (mask + feature + GN) on synthetic 64-beam 120k-pt scans.

One step = one new frame for each of B sequences in flight on this GPU, through the whole hot
path (BASELINE.json north_star):
  * scene-flow dynamic-point mask: GaussianMixture(2) fit + Kabsch pose + quaternion
    (PointCloudOdometry_noSeg.py:97-125)                       -> k_mask_pose         [mask streams]
  * frameFeature: ring binning, curvature, planar selection (frameFeature.cpp:45-123)
                                                               -> k_bin_count / k_bin_scan / k_bin_curv / k_select
  * plane table of the new frame (it is the next step's last frame)    -> k_plane_table_sorted
                                                                                      [feature stream]
  * registration of the pair (previous frame, new frame): association + 10 Gauss-Newton
    iterations + pose accumulation (lidarOdometry_onlyPC.cpp:147-252, :87-90)
                                                               -> k_associate_* / k_solve [reg stream]
  * N > 1: one RCCL all_gather of the step's per-frame 6-DoF poses (weak scaling: every rank
    owns B sequences, no other data-path collective).
Configs (BASELINE.json): default = configs[1]/[4] shape (B = 256 pairs in flight, 120k points);
--n-az 4000 = configs[4] (256k-point scans); --mask-before-features --batch 32 = configs[2]
(the features, and so the registration, see only the GMM background points).

Inputs are resident in HBM before the timed region.  After the timed region a short kernel pass
re-runs a few steps on ONE stream with per-kernel HIP events (ssf_profile_enable), so the
roofline fractions come from kernel-only durations (the timed run overlaps streams, where an
event pair also counts time spent queued behind other streams' work-groups).
`python bench.py --gpus N` without WORLD_SIZE starts N ranks itself (torch.distributed.run).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(REPO, "ssf-slam_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
F64_PEAK_TFLOPS = 78.6      # MI355X FP64 vector, spec (AMD datasheet); f64 MFMA is no faster
# HBM bytes per launch of every kernel / f64 FLOPs per k_mask_pose launch, measured with rocprofv3
# PMC passes on a serial run of this bench (tools/pmc_traffic.py, tools/pmc_f64.py); used when
# their workload config matches the run's.
TRAFFIC_JSON = os.path.join(REPO, "profiles", "r06fin_traffic.json")
# PMC traffic of the same build on the reference's own layout (--layout carla)
TRAFFIC_JSONS = {"azimuth": TRAFFIC_JSON, "carla": os.path.join(REPO, "profiles", "r06fin_carla_traffic.json")}
F64_JSON = os.path.join(REPO, "profiles", "r06fin_f64.json")
METRIC = "LiDAR front-end frames/sec (mask+feature+GN), 64-beam 120k pts, 1/2/4/8 GPUs"


def _load_profile(path, B, N, masked, layout="azimuth"):
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    cfg = t.get("config", {})
    if (cfg.get("sequences_per_gpu") != B or cfg.get("points_per_frame") != N
            or bool(cfg.get("mask_before_features")) != bool(masked)
            or cfg.get("layout", "azimuth") != layout):
        return None
    return t


def _alloc_delta(mem0, mem1):
    """the caching allocator inside the timed region: device allocations (hipMalloc) and retries
    (a retry frees cached blocks and synchronises the device)"""
    return {k: int(mem1.get(k, 0)) - int(mem0.get(k, 0))
            for k in ("num_alloc_retries", "num_device_alloc", "num_device_free", "num_ooms")}


def _lib_sha16():
    """sha256[:16] of the front-end library this run loads (ties committed PMC profiles to a build)"""
    import hashlib
    from ssf import _abi
    try:
        with open(_abi.LIB_PATH, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without WORLD_SIZE in the env, bench.py starts them")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None,
                    help="sequences in flight per GPU (default 256; 1 with --consecutive)")
    ap.add_argument("--n-az", type=int, default=1875,
                    help="azimuth steps (64 x 1875 = 120k pts; 4000 -> 256k, BASELINE configs[4])")
    ap.add_argument("--rows", type=int, default=64)
    ap.add_argument("--layout", default="azimuth", choices=["azimuth", "carla"],
                    help="synthetic scan layout: azimuth-major, every ray returns (default), or the "
                         "reference's own data layout (ssf/synth.py 'carla': channel-major, no-return "
                         "rays and road points dropped, random drop-off to the same point count)")
    ap.add_argument("--solver", default="gn", choices=["gn", "ceres_lm"])
    ap.add_argument("--iters", type=int, default=None)
    ap.add_argument("--distinct", type=int, default=None,
                    help="distinct synthetic sequences (default: every sequence distinct)")
    ap.add_argument("--mask-before-features", action="store_true",
                    help="BASELINE configs[2]: features and registration on the GMM background "
                         "points only (beyond the reference, whose frameFeature sees every point)")
    ap.add_argument("--edges", action="store_true",
                    help="beyond the reference (off by default): edge features + point-to-line "
                         "blocks in the registration (north_star wording; the reference is planar)")
    ap.add_argument("--f64-inputs", action="store_true",
                    help="the mask reads float64 pos / flow (ssf_mask_pose_batch_f64: the reference's "
                         "dtype when its npz arrays are float64); the features keep the float32 cloud "
                         "(PointCloud2 carries f32).  72 B resident per point and step: use <= 30 steps")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="CPU baseline: seconds per leg (single thread, all cores, sklearn)")
    ap.add_argument("--cpu-cores", type=int, default=None,
                    help="processes of the all-cores leg (default: this job's CPU share)")
    ap.add_argument("--kernel-pass", type=int, default=3,
                    help="steps re-run on one stream with per-kernel events after the timed run")
    ap.add_argument("--serial", action="store_true", help="one stream (per-kernel timing without overlap)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N>1 rehearsal on a one-GPU box: every rank on cuda:0, gloo collectives "
                         "(the printed line is marked rehearsal; not a scaling measurement)")
    ap.add_argument("--feat-priority", type=int, default=-1,
                    help="HIP stream priority of the features/registration streams (lower = higher)")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="registration on the features stream (default: its own stream and context, so "
                         "features + plane table of step k+1 run ahead of the registration of step k)")
    ap.add_argument("--reg-after-table", action="store_true",
                    help="the registration of step k waits for step k's plane table too (before "
                         "round 4's end; it needs only the table of step k - 1)")
    ap.add_argument("--dump-poses", default=None,
                    help="save the accumulated poses after the timed steps (.npy; stream-order check)")
    ap.add_argument("--launch-check", action="store_true",
                    help="CPU-only check of the rank launch: every rank joins a gloo group, rank 0 "
                         "prints the world it sees and exits (no GPU is touched)")
    ap.add_argument("--mask-split", type=int, default=0,
                    help="work-groups per frame of the GMM fit (0: automatic, ssf_set_mask_split)")
    ap.add_argument("--ring-depth", type=int, default=4,
                    help="step buffers in the default pipeline's ring (>= 3)")
    ap.add_argument("--seq-ring", type=int, default=8,
                    help="with --consecutive / --sequences-total: step buffers in the ring (>= 3)")
    ap.add_argument("--no-chain-api", action="store_true",
                    help="with --consecutive and one sequence: one ssf_register_batch call per chained pair "
                         "(the round-4 path) instead of ssf_register_chain")
    ap.add_argument("--consecutive", type=int, default=0,
                    help="BASELINE configs[2] as written: K consecutive frame pairs of each sequence "
                         "per step (mask of K frames in one launch, masked features, K chained "
                         "registrations); --batch sequences side by side")
    ap.add_argument("--sequences-total", type=int, default=0,
                    help="BASELINE configs[3] as written: this many sequences in total, sharded over "
                         "the --gpus ranks (strong scaling), --consecutive K (default 32) frames of "
                         "each per step, chained registrations, one pose all-gather at the end")
    ap.add_argument("--kabsch-warm-start", action="store_true",
                    help="with --consecutive / --sequences-total (beyond the reference): warm-start "
                         "every pair from its own SSF Kabsch pose, so all pairs of a step are "
                         "independent (two registration launches per step instead of K)")
    ap.add_argument("--timeline", action="store_true",
                    help="with --consecutive / --sequences-total: HIP events around every step's mask, "
                         "features + table and registrations on their streams; per-step start / end "
                         "times (ms from the first timed step) to stderr (diagnostic)")
    ap.add_argument("--timeline-host", action="store_true",
                    help="as --timeline, host enqueue times only (no timing events on the streams)")
    ap.add_argument("--latency", action="store_true",
                    help="BASELINE configs[1] as written: one frame pair at a time (B = 1), ms per frame")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES for this process (set before HIP starts; 0 = leave the "
                         "environment's, HIP's default 4). 8 measured the same as 4 over three "
                         "alternations (r04bq: 56.7 vs 56.6 k frames/s; 58.0 / 58.1 vs 55.4 / 57.2 k "
                         "in r04bp was box noise)")
    ap.add_argument("--no-ring", dest="ring", action="store_false",
                    help="allocate every step's plane cloud / plane table / mask outputs anew, with "
                         "cross-stream record_stream (the pipeline before round 5; A/B of the ring)")
    ap.add_argument("--stagger", type=int, default=200,
                    help="sequence b of a batch starts at frame (7 b) mod STAGGER (0: every sequence "
                         "at frame 0), so the timed steps sample the whole sequence length")
    ap.add_argument("--mask-order", default="none", choices=["none", "prev"],
                    help="dispatch order of a mask launch's frames (ssf_set_mask_schedule): 'prev' = "
                         "longest-first by the passes of the previous launch on the same mask stream "
                         "(the same sequences' frames one stream cycle earlier); outputs are unchanged")
    ap.add_argument("--mask-queue", type=int, default=-1,
                    help="mask launches as frame queues of at most this many work-groups (0: one "
                         "work-group per frame; -1: 3/4 of the device's CUs, 192 on MI355X -- "
                         "r6h: 96 / 128 / 160 / 192 / 224 / one per frame gave 59.7 / 60.8 / 61.9 / "
                         "62.3 / 60.4 / 55.6 k frames/s)")
    ap.add_argument("--mask-streams", type=int, default=3,
                    help="mask launches of consecutive steps alternate over this many streams: the "
                         "GMM of a frame depends on no other frame, so a step's slow frames overlap "
                         "the next step's mask instead of idling the other CUs")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------- rank launch
def launch_ranks(args) -> int:
    """--gpus N with no WORLD_SIZE: start N ranks of this script with torch.distributed.run as a
    child process (nothing here has touched the GPU) and return its exit code."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------------------- CPU baseline
def _cpu_share():
    """CPUs this job may use: OMP_NUM_THREADS / MAX_JOBS (the GPU box sets them to its per-GPU
    CPU share, 16; nproc there shows the whole machine), else the affinity set."""
    for k in ("OMP_NUM_THREADS", "MAX_JOBS"):
        v = os.environ.get(k)
        if v and v.isdigit() and int(v) > 0:
            return int(v)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _physical_cpus(n):
    """Up to n CPUs of this process's affinity set, at most one per physical core (SMT siblings
    skipped; sysfs topology) -> (cpus, siblings_skipped).  Falls back to the set in order."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except AttributeError:
        return list(range(n)), False
    seen, pick = set(), []
    for c in allowed:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            key = (open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip())
        except OSError:
            key = ("cpu", str(c))
        if key in seen:
            continue
        seen.add(key)
        pick.append(c)
        if len(pick) == n:
            break
    return pick, len(seen) < len(allowed)


def _run_legs(specs, seconds, cpus=None):
    """start every leg process at once (leg i pinned to cpus[i] when given); -> list of parsed
    JSON results"""
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    procs = []
    for i, (leg, seq, extra) in enumerate(specs):
        cmd = [sys.executable, "-m", "oracle.cpu_leg", leg, "--seq", str(seq), "--seconds",
               str(seconds), *extra]
        if cpus and leg != "sklearn":
            cmd += ["--cpu", str(cpus[i % len(cpus)])]
        e = dict(os.environ) if leg == "sklearn" else env
        procs.append(subprocess.Popen(cmd, cwd=REPO, env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.DEVNULL, text=True))
    out = []
    for p in procs:
        try:
            so, _ = p.communicate(timeout=seconds * 4 + 120)
            out.append(json.loads(so.strip().splitlines()[-1]))
        except Exception as e:  # a failed leg is reported, never silently dropped
            p.kill()
            out.append(dict(frames=0, seconds=0.0, error=str(e)))
    return out


def cpu_baseline(args):
    """The CPU restatement of the reference path (oracle/ssf_oracle.c), timed on this host
    BEFORE the GPU is touched, on a bounded sample of the same workload: one leg single-threaded,
    one with a process per core of this job's CPU share (one sequence each), and the reference's
    own third-party mask call (sklearn GaussianMixture) for the mask stage alone."""
    iters = args.iters or (10 if args.solver == "gn" else 8)
    extra = ["--rows", str(args.rows), "--n-az", str(args.n_az), "--solver", args.solver,
             "--iters", str(iters), "--layout", args.layout]
    share = args.cpu_cores or _cpu_share()
    cpus, smt = _physical_cpus(share)
    cores = len(cpus)
    T = args.cpu_seconds
    single = _run_legs([("oracle", 0, extra)], T, cpus[:1])[0]
    many = _run_legs([("oracle", s, extra) for s in range(cores)], T, cpus)
    skl = _run_legs([("sklearn", 0, ["--rows", str(args.rows), "--n-az", str(args.n_az),
                                     "--layout", args.layout])], T)[0]
    rate = lambda r: r["frames"] / r["seconds"] if r.get("seconds") else 0.0
    agg = sum(rate(r) for r in many)
    N = args.rows * args.n_az
    work = f"mask+features+plane table+{args.solver} x{iters}"
    return dict(
        value=agg, unit="frames/s", cores=cores, kind="port",
        sample=f"{sum(r['frames'] for r in many)} frames of {args.rows}-beam {N}-pt synthetic "
               f"scans ({work}) through oracle/ssf_oracle.c (gcc -O3 -ffp-contract=off), {cores} "
               f"processes x 1 thread, each pinned to its own physical core (SMT siblings "
               f"{'present in the affinity set and left idle' if smt else 'not present'}) "
               f"(one sequence each, {T:.0f} s each, concurrent)",
        legs={
            "single_thread": dict(value=rate(single), cores=1, frames=single.get("frames"),
                                  seconds=single.get("seconds"), kind="port"),
            "all_cores": dict(value=agg, cores=cores, frames=sum(r["frames"] for r in many),
                              per_process=[round(rate(r), 3) for r in many], cpus=cpus,
                              smt_siblings_in_affinity_set=smt, kind="port"),
            "sklearn_mask_only": dict(value=rate(skl), cores="BLAS default",
                                      frames=skl.get("frames"), seconds=skl.get("seconds"),
                                      kind="third-party (sklearn GaussianMixture + numpy Kabsch)",
                                      note=skl.get("skipped") or f"sklearn {skl.get('sklearn')}, "
                                      "mask + pose only (no features, no registration)"),
        })


# ---------------------------------------------------------------------------- data
def stagger_starts(args, B):
    """First frame of each sequence of the batch: sequence b starts at frame
    (7 b) mod --stagger, so one step's B frames sit at B different points of their trajectories
    and a short timed window samples the whole sequence length the reference replays
    (PointCloudOdometry_noSeg.py:58-66 walks every frame of DATASET_PATH); --stagger 0 starts
    every sequence at frame 0 (the lines before round 6)."""
    P = int(getattr(args, "stagger", 0) or 0)
    return [(7 * b) % P for b in range(B)] if P > 0 else None


def frame_window(args, B, n_frames):
    st = stagger_starts(args, B) or [0]
    return {"stagger": int(getattr(args, "stagger", 0) or 0), "first_frame_min": min(st),
            "first_frame_max": max(st), "frames_per_sequence": n_frames,
            "timed_frames": [args.warmup, args.warmup + args.steps]}


def make_data(args, dev, n_frames, rank, batch=None):
    """[n_frames] batches of B frames: pos/flow packed [B*N, 3] f32, resident in HBM.  Sequence
    b of rank r is synth sequence r * 100000 + (b mod distinct), ray-cast on the GPU
    (ssf.synth.BatchScanner: synth.scan's scenes and sensor, one ray per thread)."""
    import torch
    from ssf import synth
    B = batch or args.batch
    S = max(1, min(args.distinct or B, B))
    N = args.rows * args.n_az
    scanner = synth.BatchScanner([rank * 100000 + (b % S) for b in range(B)], n_frames,
                                 n_rows=args.rows, n_az=args.n_az, device=dev, layout=args.layout,
                                 start=stagger_starts(args, B))
    out = []
    for k in range(n_frames):
        pos = torch.empty((B * N, 3), dtype=torch.float32, device=dev)
        flow = torch.empty((B * N, 3), dtype=torch.float32, device=dev)
        scanner.frame(k, pos, flow)
        if getattr(args, "f64_inputs", False):   # the mask's float64 copies (same values)
            out.append((pos, flow, pos.double(), flow.double()))
        else:
            out.append((pos, flow))
    torch.cuda.synchronize(dev)
    return out


# ---------------------------------------------------------------------------- pipeline
class Pipeline:
    """Per-step launches of the hot path on (mask, features, registration) streams."""

    def __init__(self, args, dev, B, N, iters, world):
        import torch
        import ssf
        self.args, self.dev, self.B, self.N, self.world = args, dev, B, N, world
        self.fe_mask = ssf.Frontend(args.rows, device=dev.index)
        self.fe_feat = ssf.Frontend(args.rows, device=dev.index, solver=args.solver, max_iter=iters)
        self.fe_mask.reserve(B, N)
        self.fe_mask.mask_split(args.mask_split)
        self.fe_feat.reserve(B, N)
        n_ms = 1 if args.serial else max(1, args.mask_streams)
        self.s_masks = [torch.cuda.Stream(dev) for _ in range(n_ms)]
        # the registration chain is serial across steps: its streams get the higher priority so
        # the mask launches (independent frames) fill the CUs it leaves free
        self.s_feat = self.s_masks[0] if args.serial else torch.cuda.Stream(dev, priority=args.feat_priority)
        # registration on its own stream and context: features + plane table of step k + 1 do
        # not wait for the registration of step k (it only needs the plane table of its frames)
        pipelined = not args.serial and args.pipeline
        self.s_reg = torch.cuda.Stream(dev, priority=args.feat_priority) if pipelined else self.s_feat
        self.fe_reg = self.fe_feat
        if pipelined:
            self.fe_reg = ssf.Frontend(args.rows, device=dev.index, solver=args.solver, max_iter=iters)
            self.fe_reg.reserve(B, N)
        self.pose_rel = ssf.identity_poses(B, dev)
        self.pose_abs = ssf.identity_poses(B, dev)
        self.last = self.last_table = None
        self.last_e = self.last_etable = None
        # round 5: a ring of per-step output buffers (plane cloud, plane table, background mask),
        # allocated once (in the warmup) instead of ~2 GB of allocations per step with
        # cross-stream record_stream; slot k % RING is written by step k and read by the
        # registrations of steps k and k + 1, so step k waits for the registration of step
        # k + 2 - RING before it overwrites the slot
        self.ring, self.reg_done, self.feat_done = [], {}, {}
        self.RING = max(3, args.ring_depth)
        if args.ring:
            self.slot(self.RING - 1)                          # every slot now, not in the timed region
        self.records = []           # per timed step: the pose record this rank contributed
        self.gathered = []          # per timed step: the all-gathered records of every rank
        self.snaps = []             # (pose snapshot on s_reg, mask out, its streams) until exchange()
        # the per-step pose snapshots of N > 1 (exchange()), allocated here, not per step
        self.snapbuf = (torch.empty((args.steps, B, 7), dtype=torch.float64, device=dev)
                        if world > 1 else None)
        self.ev = {k: [] for k in ("mask", "feat", "table", "reg")}
        # --mask-order prev: per mask stream, the previous launch's pose out and the order buffers
        # (int32 permutation the kernel reads; sort scratch), all on that stream
        if args.mask_queue < 0:              # 3/4 of the CUs (one mask work-group fills a CU)
            args.mask_queue = 3 * torch.cuda.get_device_properties(dev).multi_processor_count // 4
        self.mask_prev = [None] * len(self.s_masks)
        self.mask_ord = [(torch.empty(B, dtype=torch.float64, device=dev), torch.empty(B, dtype=torch.int64, device=dev),
                          torch.empty(B, dtype=torch.int32, device=dev)) for _ in self.s_masks]

    RING = 4

    def slot(self, k):
        import torch
        i = k % self.RING
        while len(self.ring) <= i:
            B, N, d = self.B, self.N, self.dev
            T = B * N
            self.ring.append(dict(
                bg=torch.empty(T, dtype=torch.uint8, device=d),
                plane=torch.empty((T, 4), dtype=torch.float32, device=d),
                count=torch.empty(B, dtype=torch.int32, device=d),
                table=(torch.empty((T, 3), dtype=torch.float32, device=d),
                       torch.empty(T, dtype=torch.uint8, device=d),
                       torch.empty((T, 4), dtype=torch.float32, device=d),
                       torch.empty(T, dtype=torch.int32, device=d),
                       torch.empty((T, 4), dtype=torch.float32, device=d),
                       torch.empty(T, dtype=torch.int32, device=d))))
            if self.args.edges:             # the edge cloud and its line table (--edges)
                self.ring[-1].update(edge=torch.empty((T, 4), dtype=torch.float32, device=d),
                                     ecount=torch.empty(B, dtype=torch.int32, device=d),
                                     etable=(torch.empty((T, 6), dtype=torch.float32, device=d),
                                             torch.empty(T, dtype=torch.uint8, device=d)))
        return self.ring[i]

    def contexts(self):
        return [self.fe_mask, self.fe_feat] + ([self.fe_reg] if self.fe_reg is not self.fe_feat else [])

    def step(self, k, batches, off, h_off, timing, streams=None, want_stats=False):
        import torch
        a = self.args
        pos, flow = batches[k][:2]
        mpos, mflow = batches[k][2:4] if len(batches[k]) == 4 else (pos, flow)   # --f64-inputs
        s_mask, s_feat, s_reg = streams or (self.s_masks[k % len(self.s_masks)], self.s_feat, self.s_reg)
        mk = lambda: torch.cuda.Event(enable_timing=True)
        # the kernel pass allocates its own; --no-ring: the per-step allocations before round 5
        ring = self.slot(k) if streams is None and a.ring else None
        if ring is not None:
            # the slot's previous readers: the features (mask before features) of step k - RING,
            # the registrations of steps k - RING and k + 1 - RING
            if a.mask_before_features and (k - self.RING) in self.feat_done:
                s_mask.wait_event(self.feat_done.pop(k - self.RING))
            if (k + 1 - self.RING) in self.reg_done:
                s_feat.wait_event(self.reg_done.pop(k + 1 - self.RING))
        with torch.cuda.stream(s_mask):
            m0, m1 = mk(), mk()
            m0.record(s_mask)
            si = k % len(self.s_masks)
            if a.mask_order == "prev" or a.mask_queue > 0:
                order = None
                prev = self.mask_prev[si]
                if a.mask_order == "prev" and prev is not None and streams is None:
                    vals, idx, order = self.mask_ord[si]
                    torch.sort(prev[:, 25], descending=True, stable=True, out=(vals, idx))
                    order.copy_(idx)
                self.fe_mask.mask_schedule(order, a.mask_queue)
            out, bg = self.fe_mask.mask_pose(mpos, mflow, off, h_off, mode="gmm", want_mask=True,
                                             out=None if ring is None else (
                                                 torch.empty((self.B, 32), dtype=torch.float64, device=self.dev),
                                                 ring["bg"]))
            m1.record(s_mask)
            if streams is None:
                self.mask_prev[si] = out
            if a.mask_order == "prev" or a.mask_queue > 0:
                self.fe_mask.mask_schedule()
        keep = None
        if a.mask_before_features:          # configs[2]: the features wait for the mask
            if s_feat is not s_mask:
                s_feat.wait_event(m1)
                if ring is None:
                    bg.record_stream(s_feat)
            keep = bg
        eb = etable = None
        with torch.cuda.stream(s_feat):
            es = [mk() for _ in range(3)]
            es[0].record(s_feat)
            if a.edges:                     # beyond the reference: edge features as well
                pb, eb = self.fe_feat.extract_features_batch(
                    pos, off, h_off, max_points=self.N, keep=keep,
                    out=None if ring is None else (ring["plane"], ring["count"], ring["edge"], ring["ecount"]))
            else:
                pb = self.fe_feat.extract_planes_batch(pos, off, h_off, max_points=self.N, keep=keep,
                                                       out=None if ring is None else (ring["plane"], ring["count"]))
            es[1].record(s_feat)
            table = self.fe_feat.plane_table(pb, out=None if ring is None else ring["table"])
            if a.edges:
                etable = self.fe_feat.edge_table(eb, out=None if ring is None else ring["etable"])
            es[2].record(s_feat)
        if s_reg is not s_feat:
            # registration k needs the plane cloud of step k and the TABLE OF STEP k - 1 (on s_feat
            # before this step's features): it waits for the features only and runs beside this
            # step's table, which registration k + 1 gets through its own wait (same stream order)
            s_reg.wait_event(es[2] if a.reg_after_table else es[1])
            # the plane batch and its table are read on s_reg in this step and the next: keep
            # the caching allocator from handing their blocks to s_feat until s_reg is done
            extra = (eb.xyzi, eb.count, *etable) if a.edges else ()
            if ring is None:                # ring buffers are guarded by the events above instead
                for t in (pb.xyzi, pb.count, *table.tensors(), *extra):
                    t.record_stream(s_reg)
        stats = None
        with torch.cuda.stream(s_reg):
            r0, r1 = mk(), mk()
            r0.record(s_reg)        # after the wait: registration time excludes queueing on s_feat
            if self.last is not None:
                edges = (self.last_e, self.last_etable, eb) if a.edges else None
                res = self.fe_reg.register(self.last, self.last_table, pb, self.pose_rel, self.pose_abs,
                                           want_nlog=want_stats, edges=edges)
                if want_stats:
                    stats = (res["ncorr"], res["nlog"])
            r1.record(s_reg)
            snap = None
            if self.world > 1 and timing:     # step-k poses, on s_reg, into the preallocated records
                snap = self.snapbuf[len(self.snaps)]
                snap.copy_(self.pose_abs)
        if ring is not None:
            self.reg_done[k] = r1
            if a.mask_before_features:
                self.feat_done[k] = es[1]
        self.last, self.last_table = pb, table
        self.last_e, self.last_etable = eb, etable
        if self.world > 1 and timing:   # for the deferred exchange (exchange()): no per-step wait
            self.snaps.append((snap, out, s_mask, s_reg))
        if timing:
            self.ev["mask"].append((m0, m1)); self.ev["feat"].append((es[0], es[1]))
            self.ev["table"].append((es[1], es[2])); self.ev["reg"].append((r0, r1))
        return dict(out=out, bg=bg, pb=pb, stats=stats)

    def exchange(self):
        """The one exchange step (N > 1): every step's per-frame 6-DoF pose records of every rank
        in ONE all-gather (RCCL), after the last step -- SURVEY §8(e) "once per batch or at the
        end of a sequence"; no step of the pipeline waits for it."""
        from ssf import dist as sd
        if not self.snaps:
            return
        import torch
        cur = torch.cuda.current_stream(self.dev)
        for s in {id(x[2]): x[2] for x in self.snaps}.values():
            cur.wait_stream(s)
        cur.wait_stream(self.s_reg)
        recs = []
        for snap, out, _, _ in self.snaps:
            snap.record_stream(cur)
            out.record_stream(cur)
            recs.append(sd.pose_record(snap, out))
        self.records.extend(recs)
        g = sd.gather_pose_records(recs)                 # [K, world * B, 14]
        self.gathered.extend(list(g))
        self.snaps = []


def kernel_pass(pipe, batches, off, h_off, ks, rows, row_start, row_end):
    """Steps ks re-run on ONE stream with per-kernel HIP events: kernel-only durations plus the
    algorithmic byte counts of the same launches (SURVEY §8(d) per-unit figures)."""
    import torch
    import ssf
    s = torch.cuda.Stream(pipe.dev)
    s.wait_stream(torch.cuda.current_stream(pipe.dev))
    ctxs = pipe.contexts()
    pipe.last = pipe.last_table = None
    pipe.last_e = pipe.last_etable = None
    for c in ctxs:
        c.kernel_times()          # drop anything recorded earlier
        c.profile(True)
    B, N = pipe.B, pipe.N
    acc = dict(points=0, chunks=0, kept=0, in_range=0, plane=0, plane_reg=0, corr_evals=0, corr=0, mask_passes=[])
    with torch.cuda.stream(s):
        for i, k in enumerate(ks):
            r = pipe.step(k, batches, off, h_off, False, streams=(s, s, s), want_stats=True)
            # counts for the byte model (profiling paused: this extra launch is not timed)
            pipe.fe_feat.profile(False)
            keep = r["bg"] if pipe.args.mask_before_features else None
            _, _, roff, _ = pipe.fe_feat.extract_planes_batch(batches[k][0], off, h_off, max_points=N,
                                                              debug=True, keep=keep)
            pipe.fe_feat.profile(True)
            roff = roff.to(torch.int64)
            acc["points"] += B * N
            acc["chunks"] += B * ((N + 2047) // 2048)
            acc["kept"] += int(roff[:, -1].sum())
            acc["in_range"] += int((roff[:, rows - row_end] - roff[:, row_start]).sum())
            acc["plane"] += int(r["pb"].count.sum())
            acc["mask_passes"].append(r["out"][:, 25])
            if r["stats"] is not None:
                nc, nl = r["stats"]
                nc = nc.to(torch.int64).clamp(min=0)
                acc["corr"] += int(nc.sum())
                acc["corr_evals"] += int((nc * (nl.to(torch.int64) + 1)).sum())
                acc["plane_reg"] += int(r["pb"].count.sum())
    s.synchronize()
    times = {}
    for c in ctxs:
        for name, (n, ms) in c.kernel_times().items():
            a, b = times.get(name, (0, 0.0))
            times[name] = (a + n, b + ms)
        c.profile(False)
    return times, acc


def rooflines(times, acc, B, N, layout="azimuth"):
    """{kernel: launches, ms per launch, algorithmic bytes per launch, GB/s, fraction of HBM
    peak}.  The byte totals cover exactly the launches the pass profiled (features, table and
    mask: every pass step; association and solve: the steps that had a last frame)."""
    import torch
    passes = float(torch.cat(acc["mask_passes"]).mean()) if acc["mask_passes"] else 0.0
    n_mask = len(acc["mask_passes"])
    model = {   # DESIGN.md §5 / SURVEY §8(d) per-unit figures
        "k_mask_pose": B * N * (24.0 * passes + 1.0) * n_mask,     # [flow,xyz] f32 per pass + mask
        "k_mask_pose_f64": B * N * (48.0 * passes + 1.0) * n_mask,  # [flow,xyz] f64 per pass + mask
        "k_bin_count": 13.0 * acc["points"],                        # xyz read, row id written
        # the stable partition fused with the 11-tap curvature: xyz + row id read once per point
        # (the halo's re-reads of neighbouring chunks are L2 hits, not algorithmic), per kept
        # point its input index (4 B) and candidate flag byte written at its ring position
        "k_bin_curv": 13.0 * acc["points"] + 5.0 * acc["kept"],
        # round 4, the single-read stage: xyz read once (12 B), a u16 chunk position per point
        # (2 B) written, per 2048-point chunk its row counts (256 B) and two bit planes (512 B)
        "k_feat_chunk": 14.0 * acc["points"] + 768.0 * acc["chunks"],
        # round 4: the regular-window kernel does every chunk of an unmasked 64-beam azimuth-ordered
        # frame (the bench's scans): the same bytes + its block flag; k_feat_chunk then only reads
        # the flags (its model is dropped below when this kernel ran)
        # (no u16 index: a 64-B row -> lane map per chunk instead)
        "k_feat_chunk_reg": 12.0 * acc["points"] + 833.0 * acc["chunks"],
        # the same outputs with one wave per chunk (its halo columns are L2 hits, not algorithmic)
        "k_feat_wave_reg": 12.0 * acc["points"] + 833.0 * acc["chunks"],
        # the chunks' counts and bit planes read, per plane point: its u16 position (2 B) and xyz
        # (12 B) gathered, the xyzi record written (16 B); the selections stay in LDS
        "k_feat_select": 768.0 * acc["chunks"] + 30.0 * acc["plane"],
        # flag bytes read, per plane point: its index written and read back (4 + 4 B), its ring
        # index (4 B) and xyz (12 B) gathered and the xyzi record written (16 B)
        "k_select": 1.0 * acc["kept"] + 40.0 * acc["plane"],
        # plane point read (16 B), x-sorted copy + permutation (16 + 4), normal + validity
        # (12 + 1), and the y-strip image the next pair's association stages (16 + 4)
        "k_plane_table_sorted": 69.0 * acc["plane"],
        "k_associate_lds": 64.0 * acc["plane_reg"],
        "k_associate_lds_soa": 64.0 * acc["plane_reg"],
        "k_associate_strips": 64.0 * acc["plane_reg"],
        "k_associate_strips_soa": 64.0 * acc["plane_reg"],
        "k_associate_sorted": 64.0 * acc["plane_reg"],
        "k_solve": 36.0 * acc["corr_evals"],                        # §8(d): 36 B x C per evaluation
    }
    if "k_feat_chunk_reg" in times or "k_feat_wave_reg" in times:
        model.pop("k_feat_chunk", None)
        # select reads the lane maps (and flags) and no u16 positions
        model["k_feat_select"] = 833.0 * acc["chunks"] + 28.0 * acc["plane"]
    if layout == "carla":
        # round 5, the reference's own layout (channel-major runs): k_feat_wave_run does the chunks
        # -- xyz read once (12 B), per chunk its row counts (256 B), two bit planes (512 B), the
        # rows' u16 run starts (128 B) and its flag -- after k_feat_wave_reg's probe, which reads
        # one 64-point column per chunk (768 B) and leaves; k_feat_select reads the run start of a
        # plane point's (chunk, row) (2 B) instead of a lane map
        model["k_feat_wave_run"] = 12.0 * acc["points"] + 897.0 * acc["chunks"]
        model["k_feat_wave_reg"] = 768.0 * acc["chunks"]
        model.pop("k_feat_chunk", None)
        model["k_feat_select"] = 897.0 * acc["chunks"] + 30.0 * acc["plane"]
    out = {}
    for name, (n, ms) in sorted(times.items(), key=lambda kv: -kv[1][1]):
        d = dict(launches=n, ms=ms / n)
        if name in model and ms > 0:
            bytes_per = model[name] / n
            gbs = bytes_per / (ms / n * 1e-3) / 1e9
            d.update(bytes=bytes_per, gbs=gbs, frac=gbs / HBM_PEAK_GBS)
        out[name] = d
    if "k_solve" in out:
        n = out["k_solve"]["launches"]
        out["k_solve"].update(corr_per_launch=acc["corr"] / n,
                              evaluations_per_pair=acc["corr_evals"] / max(1, acc["corr"]),
                              note="corr = valid correspondences counted on device (ncorr); "
                                   "evaluations = 1 + logged iterations (nlog)")
    for k in ("k_bin_curv", "k_feat_chunk", "k_feat_chunk_reg", "k_feat_wave_reg", "k_feat_wave_run"):
        if k in out:
            out[k]["kept_points_per_launch"] = acc["kept"] / out[k]["launches"]
    return out, passes


def latency(args):
    """BASELINE configs[1] as written: ONE 120k-point frame pair at a time, the way the
    reference's nodes see it -- PointCloudOdometry_noSeg.py:97-125 masks one frame per callback,
    frameFeature extracts one frame (frameFeature.cpp:35-139), and cloudThread registers one
    plane cloud against the previous one (lidarOdometry_onlyPC.cpp:281-311).  Per frame: the
    mask (GMM + Kabsch, automatic split: G = 8 work-groups for one frame) on one stream, and
    features -> plane table -> registration of the pair (10 GN iterations) on another; the
    frame is done when both have finished (host wall time per frame, synchronised).  `serial`
    runs the same calls on ONE stream (mask, then the chain), as a single-threaded node chain
    would.  The frame's plane table (needed only by the NEXT pair) is launched after its
    registration, so the latency is frame in -> both poses out; frame_period adds the table.
    Rank 0 prints one JSON line, value = median ms per frame (overlapped)."""
    import torch
    import ssf
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    iters = args.iters or (10 if args.solver == "gn" else 8)
    N = args.rows * args.n_az
    W, K = max(2, args.warmup), args.steps
    t_data = time.perf_counter()
    frames = make_data(args, dev, 2 * (W + K) + 2, 0, batch=1)
    t_data = time.perf_counter() - t_data
    off, h_off = ssf.frame_offsets([N], dev)
    fe_mask = ssf.Frontend(args.rows, device=0)
    fe_mask.reserve(1, N)
    fe_mask.mask_split(args.mask_split)
    fe_mask.seed(20240000)
    fe = ssf.Frontend(args.rows, device=0, solver=args.solver, max_iter=iters)
    fe.reserve(1, N)
    s_mask, s_chain = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    self_period = []

    def run(ks, serial, profile=False):
        pose_rel, pose_abs = ssf.identity_poses(1, dev), ssf.identity_poses(1, dev)
        last = last_table = None
        wall, ev = [], []
        if profile:
            for c in (fe_mask, fe):
                c.kernel_times()
                c.profile(True)
        period = []
        for k in ks:
            pos, flow = frames[k]
            sm, sc = (s_chain, s_chain) if serial else (s_mask, s_chain)
            e = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            with torch.cuda.stream(sm):
                e[0].record(sm)
                out, bg = fe_mask.mask_pose(pos, flow, off, h_off, mode="gmm", want_mask=True)
                e[1].record(sm)
            with torch.cuda.stream(sc):
                e[2].record(sc)
                pb = fe.extract_planes_batch(pos, off, h_off, max_points=N)
                e[3].record(sc)
                if last is not None:
                    fe.register(last, last_table, pb, pose_rel, pose_abs)
                e[4].record(sc)
                # the plane table of this frame is needed by the NEXT pair only: it runs after
                # this frame's pose is out, off the frame's critical path
                table = fe.plane_table(pb)
                e[5].record(sc)
            e[1].synchronize()
            e[4].synchronize()
            wall.append((time.perf_counter() - t0) * 1e3)      # both poses of the frame are out
            sc.synchronize()
            period.append((time.perf_counter() - t0) * 1e3)    # + the table for the next pair
            ev.append(e)
            last, last_table = pb, table
        kt = {}
        if profile:
            for c in (fe_mask, fe):
                for name, (n, ms) in c.kernel_times().items():
                    a, b = kt.get(name, (0, 0.0))
                    kt[name] = (a + n, b + ms)
                c.profile(False)
        stages = dict(mask=[a[0].elapsed_time(a[1]) for a in ev],
                      features=[a[2].elapsed_time(a[3]) for a in ev],
                      registration=[a[3].elapsed_time(a[4]) for a in ev[1:]],
                      plane_table=[a[4].elapsed_time(a[5]) for a in ev])
        self_period.extend(period[1:])
        return wall[1:], stages, kt      # the first frame of a run has no pair to register

    # warm up both orders, then time K frames of one sequence each way
    run(range(0, W), False)
    run(range(0, W), True)
    self_period.clear()
    wall_o, st_o, _ = run(range(W, W + K), False)
    period_o = list(self_period)
    wall_s, st_s, _ = run(range(W + K + 1, W + 2 * K + 1), True)
    _, _, kt = run(range(W, W + min(K, 8)), True, profile=True)
    med = lambda v: float(np.median(v)) if len(v) else 0.0
    kernels = {name: dict(launches=n, ms=ms / n) for name, (n, ms) in sorted(kt.items(), key=lambda x: -x[1][1])}
    cpu = None
    if not args.no_cpu_baseline:
        iters_s = ["--rows", str(args.rows), "--n-az", str(args.n_az), "--solver", args.solver, "--iters", str(iters)]
        single = _run_legs([("oracle", 0, iters_s)], args.cpu_seconds)[0]
        if single.get("seconds"):
            cpu = dict(value=single["seconds"] / max(1, single["frames"]) * 1e3, unit="ms/frame", cores=1,
                       kind="port", sample=f"{single['frames']} consecutive frames of one sequence through "
                                           "oracle/ssf_oracle.c (mask + features + plane table + registration), "
                                           "one thread")
    line = {
        "metric": "LiDAR front-end latency per frame pair (mask+feature+GN), 64-beam 120k pts, 1 GPU",
        "value": med(wall_o), "unit": "ms/frame", "n_gpus": 1, "steps": K, "warmup": W,
        "ms_per_step": med(wall_o), "higher_is_better": False, "scaling": "none", "vs_baseline": None,
        "dtype": "f32 features / f64 mask+solve",
        "data": "synthetic (seeded ray-cast 64-beam scans, ssf/synth.py BatchScanner; one sequence)",
        "config": {"workload": f"configs[1] as written: one {args.rows}-beam {N}-pt frame pair per step (B = 1); "
                               f"mask(GMM+Kabsch, automatic split) || features -> plane table -> {args.solver} "
                               f"x{iters}; host wall per frame, synchronised",
                   "points_per_frame": N, "solver": args.solver, "iters": iters, "batch": 1},
        "latency_ms": {"overlapped": {"median": med(wall_o), "mean": float(np.mean(wall_o)),
                                      "p90": float(np.percentile(wall_o, 90)),
                                      "note": "frame in -> SSF pose (mask + Kabsch) and registration pose out; "
                                              "the frame's plane table (needed by the next pair) runs after"},
                       "frame_period_overlapped": {"median": med(period_o),
                                                   "note": "latency + the plane table: one frame after "
                                                           "another on one GPU, nothing pipelined across frames"},
                       "serial_one_stream": {"median": med(wall_s), "mean": float(np.mean(wall_s)),
                                             "p90": float(np.percentile(wall_s, 90))}},
        "stage_event_ms": {k: med(v) for k, v in st_o.items()},
        "stage_event_ms_serial": {k: med(v) for k, v in st_s.items()},
        "kernels": kernels, "cpu_baseline": cpu, "data_gen_s": round(t_data, 2),
    }
    print(json.dumps(line), flush=True)


def _init_dist(args, world, rank, dev):
    """process group for N > 1 (RCCL, or gloo for a one-GPU rehearsal) -> backend name or None"""
    import torch.distributed as dist
    if world <= 1:
        return None
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    backend = "gloo" if args.rehearse_one_gpu else "nccl"
    if backend == "gloo":
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    if dist.get_world_size() != args.gpus:
        sys.exit(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    return backend


def sequences(args, world=1, rank=0, local=0):
    """Whole sequences, K consecutive frames of each per step.
    * BASELINE configs[2] as written (--consecutive K, one GPU): the PointCloudOdometry_noSeg.py
      path with the scene-flow mask applied before the features, K consecutive frame pairs of
      each of --batch sequences per step.
    * BASELINE configs[3] as written (--sequences-total S, 1..8 ranks): a FIXED set of S
      sequences sharded over the ranks (ssf.dist.sequence_shard: one per GPU at 8 GPUs, like one
      launch graph per CARLA sequence, run_noSeg.launch:4,15-16), every rank running its own
      sequences' frames; one deferred all-gather of the per-frame 6-DoF pose records at the end
      (RCCL over xGMI).  Strong scaling: the total work is the same at every N.  The reference's
      wiring (frameFeature sees every point, the mask runs beside it) unless --mask-before-features.
    One step = the next K frames of every owned sequence: one mask launch (GMM + Kabsch) for the
    B x K frames, features + plane table of them in one launch each, then the registrations:
    chained (default; the warm start of pair k is the solution of pair k - 1,
    lidarOdometry_onlyPC.cpp:164-169,251-252), K launches of B pairs; or, with
    --kabsch-warm-start (beyond the reference), every pair warm-started from its own SSF Kabsch
    pose, which the mask launch already produced (on the SSF path the reference publishes that pose
    itself, lidarOdometry.cpp:145-159), so the B x K pairs are independent: two launches per step.
    Masks of consecutive steps alternate over --mask-streams streams; registrations of step j
    overlap the mask of step j + 1.  Rank 0 prints one JSON line."""
    import torch
    import torch.distributed as dist
    import ssf
    from ssf import synth
    from ssf import dist as sd
    strong = args.sequences_total > 0
    if args.rehearse_one_gpu:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = _init_dist(args, world, rank, dev)
    K = args.consecutive or 32
    if strong:
        shard = list(sd.sequence_shard(args.sequences_total, world, rank))
        seeds = shard                         # a sequence's data does not depend on N
        masked = bool(args.mask_before_features)
    else:
        seeds = list(range(args.batch or 1))
        masked = True                         # configs[2] as written: mask before features
    B = len(seeds)
    iters = args.iters or (10 if args.solver == "gn" else 8)
    N = args.rows * args.n_az
    W, S = max(1, args.warmup), args.steps
    n_steps = W + S
    per_step_bytes = K * B * N * 24
    if per_step_bytes * n_steps > 120e9:
        sys.exit(f"bench.py: {n_steps} steps x {K} x {B} frames of {N} points need "
                 f"{per_step_bytes * n_steps / 1e9:.0f} GB resident; lower --batch / --consecutive")
    t_data = time.perf_counter()
    # frame 0 of every sequence (the prologue), then per step K frames, frame-major:
    # buffer index kk * B + b holds frame j K + kk + 1 of sequence b
    scanner = synth.BatchScanner(seeds, K * n_steps + 1, n_rows=args.rows, n_az=args.n_az, device=dev,
                                 layout=args.layout)
    pro = (torch.empty((B * N, 3), dtype=torch.float32, device=dev),
           torch.empty((B * N, 3), dtype=torch.float32, device=dev))
    scanner.frame(0, *pro)
    steps = []
    for j in range(n_steps):
        pos = torch.empty((K * B * N, 3), dtype=torch.float32, device=dev)
        flow = torch.empty_like(pos)
        for kk in range(K):
            scanner.frame(j * K + kk + 1, pos[kk * B * N:(kk + 1) * B * N], flow[kk * B * N:(kk + 1) * B * N])
        steps.append((pos, flow))
    torch.cuda.synchronize(dev)
    t_data = time.perf_counter() - t_data
    off1, h1 = ssf.frame_offsets([N] * B, dev)
    offK, hK = ssf.frame_offsets([N] * (K * B), dev)
    fe_mask = ssf.Frontend(args.rows, device=dev.index)
    fe_mask.reserve(K * B, N)
    # the automatic split fills the chip with ONE launch (slots / frames parts per frame); here
    # the masks of --mask-streams consecutive steps are in flight together, so each launch gets
    # its share: slots / (streams x frames) (32 frames, 3 streams: 2 parts; 256 frames: 1)
    n_ms = max(1, args.mask_streams)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    g_split = args.mask_split or max(1, cus // (n_ms * K * B))
    fe_mask.mask_split(g_split)
    fe_mask.seed(20240000 + (shard[0] if strong and shard else 0))
    fe_feat = ssf.Frontend(args.rows, device=dev.index, solver=args.solver, max_iter=iters)
    fe_feat.reserve(K * B, N)
    fe_reg = ssf.Frontend(args.rows, device=dev.index, solver=args.solver, max_iter=iters)
    fe_reg.reserve(K * B, N)
    s_masks = [torch.cuda.Stream(dev) for _ in range(n_ms)]
    s_feat = torch.cuda.Stream(dev, priority=args.feat_priority)
    s_reg = torch.cuda.Stream(dev, priority=args.feat_priority)
    rel, ab = ssf.identity_poses(B, dev), ssf.identity_poses(B, dev)
    kws = args.kabsch_warm_start

    def view(pb, table, a, b=None):
        """frames of buffer slots [a, b) as a PlaneBatch (the table arrays are shared: they are
        indexed by the frames' point offsets)"""
        b = a + 1 if b is None else b
        return ssf.PlaneBatch(pb.xyzi, pb.count[a * B:b * B], pb.off[a * B:b * B + 1],
                              pb.h_off[a * B:b * B + 1], pb.max_points), table

    def warm_start(out, dst):
        """the SSF Kabsch poses [t, q] of mask_pose -> registration warm starts [q, t] written into
        dst (identity where the mask reported a failure)"""
        dst[:, 0:4].copy_(out[:, 3:7])
        dst[:, 4:7].copy_(out[:, 0:3])
        bad = out[:, 16] != 0
        dst[:, 0:3].masked_fill_(bad.unsqueeze(1), 0.0)
        dst[:, 3].masked_fill_(bad, 1.0)
        dst[:, 4:7].masked_fill_(bad.unsqueeze(1), 0.0)

    # a ring of step buffers (mask output and background, plane cloud, plane table), allocated
    # here instead of per step: slot j % SR holds step j's; its last reader is the registration of
    # step j + 1, so step j waits for the registration of step j + 1 - SR before overwriting it.
    # The per-step pose records go to preallocated [steps, K, B, 7] arrays.
    SR = max(3, args.seq_ring)
    T_ = K * B * N
    ring = [dict(out=torch.empty((K * B, 32), dtype=torch.float64, device=dev),
                 bg=torch.empty(T_, dtype=torch.uint8, device=dev),
                 plane=torch.empty((T_, 4), dtype=torch.float32, device=dev),
                 count=torch.empty(K * B, dtype=torch.int32, device=dev),
                 table=(torch.empty((T_, 3), dtype=torch.float32, device=dev),
                        torch.empty(T_, dtype=torch.uint8, device=dev),
                        torch.empty((T_, 4), dtype=torch.float32, device=dev),
                        torch.empty(T_, dtype=torch.int32, device=dev),
                        torch.empty((T_, 4), dtype=torch.float32, device=dev),
                        torch.empty(T_, dtype=torch.int32, device=dev)))
            for _ in range(SR)]
    rec_rel = torch.empty((n_steps, K, B, 7), dtype=torch.float64, device=dev)
    rec_m = torch.empty((n_steps, K, B, 7), dtype=torch.float64, device=dev)
    reg_done = {}

    # prologue: frame 0 -> the first last frames (and its Kabsch pose: pair (0, 1)'s warm start)
    with torch.cuda.stream(s_feat):
        out0, bg0 = fe_mask.mask_pose(pro[0], pro[1], off1, h1, mode="gmm", want_mask=True)
        pb0 = fe_feat.extract_planes_batch(pro[0], off1, h1, max_points=N, keep=bg0 if masked else None)
        last = (pb0, fe_feat.plane_table(pb0))
    torch.cuda.synchronize(dev)
    prev_out = out0
    records = []

    tl = []                                   # --timeline: per step, (phase, start, end) events

    def ev(stream):
        if args.timeline_host:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e

    def step(j, timing):
        nonlocal last, prev_out
        pos, flow = steps[j]
        sm = s_masks[j % len(s_masks)]
        slot = ring[j % SR]
        if (j + 1 - SR) in reg_done:                        # the slot's last reader is done
            prev = reg_done.pop(j + 1 - SR)
            sm.wait_event(prev)
            s_feat.wait_event(prev)
        rec = {} if (timing and (args.timeline or args.timeline_host)) else None
        hst = [time.perf_counter()] if rec is not None else None   # host enqueue times
        with torch.cuda.stream(sm):
            if rec is not None:
                rec["mask"] = [ev(sm)]
            out, bg = fe_mask.mask_pose(pos, flow, offK, hK, mode="gmm", want_mask=True,
                                        out=(slot["out"], slot["bg"]))
            if rec is not None:
                hst.append(time.perf_counter())
                rec["mask"].append(ev(sm))
            mrec = rec_m[j]
            mrec.copy_(out[:, 0:7].view(K, B, 7))           # the SSF poses, on their stream
            done = torch.cuda.Event()
            done.record(sm)
        if masked:                                          # configs[2]: the features wait for the mask
            s_feat.wait_event(done)
        with torch.cuda.stream(s_feat):
            if rec is not None:
                hst.append(time.perf_counter())
                rec["feat"] = [ev(s_feat)]
            pb = fe_feat.extract_planes_batch(pos, offK, hK, max_points=N, keep=bg if masked else None,
                                              out=(slot["plane"], slot["count"]))
            table = fe_feat.plane_table(pb, out=slot["table"])
            tdone = torch.cuda.Event()
            tdone.record(s_feat)
            if rec is not None:
                rec["feat"].append(ev(s_feat))
        s_reg.wait_event(tdone)
        if kws:
            s_reg.wait_event(done)
        with torch.cuda.stream(s_reg):
            if rec is not None:
                hst.append(time.perf_counter())
                rec["reg"] = [ev(s_reg)]
            (lpb, ltab) = last
            if kws:
                # pair (slot kk - 1 -> slot kk) starts from the Kabsch pose of frame kk - 1
                ws = rec_rel[j].view(K * B, 7)
                warm_start(prev_out, ws[:B])
                if K > 1:
                    warm_start(out[:(K - 1) * B], ws[B:])
                fe_reg.register(lpb, ltab, view(pb, table, 0)[0], ws[:B])
                if K > 1:
                    fe_reg.register(*view(pb, table, 0, K - 1), view(pb, table, 1, K)[0], ws[B:])
                rel_k = rec_rel[j]
            elif B == 1 and not args.no_chain_api:
                # one sequence: the boundary pair (the previous step's last frame -> frame 0) by
                # ssf_register_batch, then the K - 1 pairs inside this step's batch by ONE
                # ssf_register_chain call (each link reads the previous solution in place: no
                # per-pair copy launches, no per-pair host calls)
                seq = rec_rel[j].view(K, 7)
                seq[0:1].copy_(rel)
                fe_reg.register(lpb, ltab, view(pb, table, 0)[0], seq[0:1], ab)
                if K > 1:
                    ch = fe_reg.register_chain(view(pb, table, 0, K)[0], table, seq[0], pose_abs_init=ab,
                                               out=seq[1:])
                    ab.copy_(ch["pose_abs_seq"][-1:])
                rel.copy_(seq[K - 1:K])
                rel_k = rec_rel[j]
            else:
                for kk in range(K):
                    cur = view(pb, table, kk)
                    fe_reg.register(lpb, ltab, cur[0], rel, ab)
                    rec_rel[j][kk].copy_(rel)
                    (lpb, ltab) = cur
                rel_k = rec_rel[j]
            rdone = torch.cuda.Event()
            rdone.record(s_reg)
            reg_done[j] = rdone
            records.append((rel_k, mrec, sm))                # (warmup records are dropped)
            if rec is not None:
                rec["reg"].append(ev(s_reg))
                hst.append(time.perf_counter())
                rec["host"] = hst
                tl.append(rec)
        last = view(pb, table, K - 1)
        prev_out = out[(K - 1) * B:]
        return out

    for j in range(W):
        step(j, False)
    # the end-of-run path once on the warmup records (first launches load their kernels: the
    # timed region must not pay that), then only timed records
    for s in (*s_masks, s_reg):
        torch.cuda.current_stream(dev).wait_stream(s)
    warm = torch.cat([torch.cat([r, m], 2) for r, m, _ in records], 0)
    if world > 1:
        sd.gather_sequence_records(warm, args.sequences_total)
    del warm
    records.clear()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    mem0 = torch.cuda.memory_stats(dev)
    t0 = time.perf_counter()
    for j in range(W, W + S):
        step(j, True)
    # per timed frame: the registration pose [q, t] and the SSF Kabsch pose [t, q] -> [F, B, 14]
    cur = torch.cuda.current_stream(dev)
    for s in (*s_masks, s_reg):
        cur.wait_stream(s)
    mine = torch.cat([torch.cat([r, m], 2) for r, m, _ in records], 0)
    gathered = None
    if world > 1:                  # the one exchange: every timed frame's records, one all-gather
        gathered = sd.gather_sequence_records(mine, args.sequences_total)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    allocator = _alloc_delta(mem0, torch.cuda.memory_stats(dev))
    if tl and rank == 0:
        z = tl[0]["mask"][0]
        h0 = tl[0]["host"][0]
        for j, rec in enumerate(tl):
            hs = rec.pop("host")
            print("timeline step %d: " % j + ("" if args.timeline_host else "  ".join(
                "%s %.3f-%.3f" % (k, z.elapsed_time(a), z.elapsed_time(b)) for k, (a, b) in rec.items()))
                + "  host(mask,masked,feat,reg,end) " + " ".join("%.3f" % ((h - h0) * 1e3) for h in hs),
                file=sys.stderr)
    gather_ok = None
    finite = bool(torch.isfinite(mine).all())
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if backend == "gloo" else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        gather_ok = bool(torch.equal(gathered[:, shard[0]:shard[-1] + 1].cpu(), mine.cpu())) if shard else True
        flag = torch.tensor([1 if gather_ok and finite else 0], dtype=torch.int32,
                            device="cpu" if backend == "gloo" else dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        gather_ok = bool(flag.item())
    total_seq = args.sequences_total if strong else B
    frames = total_seq * K * S
    ws_note = ("every pair warm-started from its own SSF Kabsch pose (beyond the reference: "
               "independent pairs, 2 launches per step)" if kws else
               f"{K} chained registrations per step (warm start = previous solution"
               + ("; the boundary pair + one ssf_register_chain call of K - 1 pairs)"
                  if B == 1 and not args.no_chain_api else "; one call per pair)"))
    if strong:
        workload = (f"configs[3] as written: {total_seq} sequences sharded over {world} GPU(s) "
                    f"(sequence_shard), {K} consecutive frames of each per step, {S} steps "
                    f"({K * S} timed frames per sequence); mask(GMM+Kabsch) "
                    f"{'before' if masked else 'beside'} features + plane table + {args.solver} "
                    f"x{iters}; {ws_note}; one all-gather of the per-frame pose records at the end")
    else:
        workload = (f"configs[2] as written: PointCloudOdometry_noSeg path, mask before features, "
                    f"{K} consecutive frame pairs of each of {B} sequence(s) per step: one mask "
                    f"launch of {K * B} frames, masked features + plane table of them, "
                    f"{args.solver} x{iters}; {ws_note}")
    line = {
        "metric": METRIC, "value": frames / elapsed, "unit": "frames/s", "n_gpus": world, "steps": S,
        "warmup": W, "ms_per_step": elapsed / S * 1e3, "higher_is_better": True,
        "scaling": "strong" if strong else "none", "vs_baseline": None,
        "dtype": "f32 features / f64 mask+solve",
        "data": f"synthetic (seeded ray-cast {args.rows}-beam scans, ssf/synth.py BatchScanner; "
                f"{total_seq} sequence(s))",
        "config": {"workload": workload, "consecutive_pairs": K, "sequences": total_seq,
                   "sequences_this_rank": B, "frames_per_sequence_timed": K * S,
                   "points_per_frame": N, "solver": args.solver, "iters": iters,
                   "mask_before_features": masked, "kabsch_warm_start": bool(kws),
                   "mask_streams": n_ms, "mask_parts_per_frame": g_split,
                   "parallelism": f"sequence-sharded x{world}",
                   "world_size_initialised": (dist.get_world_size() if world > 1 else 1),
                   "backend": backend or "none",
                   **({"rehearsal": "all ranks on one GPU, gloo"} if args.rehearse_one_gpu else {})},
        "gather_check": gather_ok, "poses_finite": finite,
        "data_gen_s": round(t_data, 2),
        "final_t_norm": float(mine[-1, :, 4:7].norm(dim=1).mean()),
        "allocator_timed_region": allocator,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.hw_queues > 0:                # before anything starts the HIP runtime
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    if args.latency:
        if args.gpus != 1 or os.environ.get("WORLD_SIZE", "1") != "1":
            sys.exit("bench.py --latency is a one-GPU, one-frame-pair measurement")
        return latency(args)
    if args.consecutive and not args.sequences_total:
        if args.gpus != 1 or os.environ.get("WORLD_SIZE", "1") != "1":
            sys.exit("bench.py --consecutive is a one-GPU measurement (configs[2]); "
                     "--sequences-total S is the multi-GPU configs[3] mode")
        return sequences(args)
    ws = os.environ.get("WORLD_SIZE")
    if ws is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(ws or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report a "
                 f"{world}-rank run as {args.gpus} GPUs")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.sequences_total and not args.launch_check:
        return sequences(args, world, rank, local)
    if args.launch_check:
        import torch
        import torch.distributed as dist
        from ssf.dist import sequence_shard
        shard = list(sequence_shard(args.sequences_total, world, rank)) if args.sequences_total else None
        if world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=rank, world_size=world)
        got = [None] * world
        if world > 1:
            dist.all_gather_object(got, dict(rank=rank, local=local, pid=os.getpid(), shard=shard))
        else:
            got = [dict(rank=0, local=local, pid=os.getpid(), shard=shard)]
        if rank == 0:
            print(json.dumps({"launch_check": True, "n_gpus": args.gpus, "world": world,
                              "ranks": got}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    if args.batch is None:
        args.batch = 256
    if args.warmup < 1:
        args.warmup = 1  # the first frame of a sequence has no last frame to register against
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)          # before anything touches the GPU

    import torch
    import torch.distributed as dist
    if args.rehearse_one_gpu:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = _init_dist(args, world, rank, dev)

    import ssf
    iters = args.iters or (10 if args.solver == "gn" else 8)
    B, N = args.batch, args.rows * args.n_az
    n_frames = args.warmup + args.steps + 1
    t_data = time.perf_counter()
    batches = make_data(args, dev, n_frames, rank)
    t_data = time.perf_counter() - t_data
    off, h_off = ssf.frame_offsets([N] * B, dev)
    pipe = Pipeline(args, dev, B, N, iters, world)
    pipe.fe_mask.seed(20240000 + rank)

    # the last warmup step takes the timed steps' code path, and the one exchange runs once, so
    # every kernel and collective the timed region uses has been loaded and set up before it
    # (HIP loads a kernel's code object on its first launch: ~50 ms for a torch copy kernel)
    for k in range(args.warmup):
        pipe.step(k, batches, off, h_off, k == args.warmup - 1)
    if world > 1:
        pipe.exchange()
    pipe.records.clear(); pipe.gathered.clear()
    pipe.ev = {k: [] for k in pipe.ev}
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    mem0 = torch.cuda.memory_stats(dev)
    t0 = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        pipe.step(k, batches, off, h_off, True)
    if world > 1:
        pipe.exchange()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # the caching allocator inside the timed region: 0 device allocations and retries with the
    # buffer ring
    allocator = _alloc_delta(mem0, torch.cuda.memory_stats(dev))
    if args.dump_poses and rank == 0:
        np.save(args.dump_poses, pipe.pose_abs.cpu().numpy())
    gather_ok = None
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if backend == "gloo" else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # every gathered record of this rank must be the pose of its own step (stream order)
        gather_ok = all(torch.equal(g[rank * B:(rank + 1) * B].cpu(), r.cpu())
                        for g, r in zip(pipe.gathered, pipe.records))
        flag = torch.tensor([1 if gather_ok else 0], dtype=torch.int32,
                            device="cpu" if backend == "gloo" else dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        gather_ok = bool(flag.item())

    # ---- overlapped-run events (context) and the kernel pass (the roofline's durations)
    def avg_ms(pairs):
        return float(np.mean([a.elapsed_time(b) for a, b in pairs])) if pairs else 0.0

    overlapped = {k: avg_ms(v) for k, v in pipe.ev.items()}
    ks = list(range(args.warmup, min(args.warmup + args.kernel_pass, n_frames)))
    kernels, passes = {}, 0.0
    if args.kernel_pass > 0:
        cfg = pipe.fe_feat.cfg
        times, acc = kernel_pass(pipe, batches, off, h_off, ks, args.rows, cfg.row_start, cfg.row_end)
        kernels, passes = rooflines(times, acc, B, N, args.layout)

    total_frames = B * args.steps * world
    value = total_frames / elapsed
    cfg_name = ("configs[2] shape, noSeg mask-before-features, B sequences x 1 frame per step "
                "(--consecutive K runs K consecutive pairs of one sequence)" if args.mask_before_features else
                "configs[4] 256k-pt stress" if args.n_az >= 4000 else
                "configs[1] shape (one 120k-pt frame pair per sequence per step)")
    line = {
        "metric": METRIC,
        "value": value, "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32 features / f64 mask+solve",
        "data": f"synthetic (seeded ray-cast 64-beam scans, ssf/synth.py, layout {args.layout}; "
                f"{min(args.distinct or B, B)} distinct sequences per rank)",
        "config": {"workload": f"{cfg_name}: {B} sequences in flight per GPU x {args.rows}-beam "
                               f"{N}-pt scans; mask(GMM+Kabsch) + "
                               f"{'masked ' if args.mask_before_features else ''}features + plane "
                               f"table + {'edge table + point-to-line + ' if args.edges else ''}"
                               f"{args.solver} x{iters}",
                   "sequences_per_gpu": B, "points_per_frame": N, "solver": args.solver,
                   "layout": args.layout,
                   "iters": iters, "mask_before_features": bool(args.mask_before_features),
                   "edges": bool(args.edges),
                   "parallelism": f"sequence-sharded x{world}",
                   "world_size_initialised": (dist.get_world_size() if world > 1 else 1),
                   "backend": backend or "none",
                   "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "0")) or None,
                   "frame_window": frame_window(args, B, n_frames),
                   "mask_schedule": {"order": args.mask_order, "queue": args.mask_queue},
                   **({"rehearsal": "all ranks on one GPU, gloo"} if args.rehearse_one_gpu else {})},
        "roofline": None, "cpu_baseline": cpu,
        "kernels": kernels, "overlapped_event_ms": overlapped,
        "mask_passes_per_frame": passes, "gather_check": gather_ok,
        "allocator_timed_region": allocator,
        "data_gen_s": round(t_data, 2), "lib_sha16": None,
    }
    if args.f64_inputs:
        line["config"]["mask_inputs"] = "float64 pos / flow (ssf_mask_pose_batch_f64), float32 features"
        line["dtype"] = "f32 features / f64 mask inputs + f64 mask+solve"
    tjson = TRAFFIC_JSONS.get(args.layout, TRAFFIC_JSON)
    traffic = None if args.edges else _load_profile(tjson, B, N, args.mask_before_features, args.layout)
    lib_sha = _lib_sha16()
    tsrc = None
    if traffic:
        # the traffic is a committed PMC measurement, not this run's: say which, and whether it
        # was measured on this very library build
        tsrc = {"traffic_source": os.path.relpath(tjson, REPO),
                "traffic_lib_sha16": traffic.get("lib_sha16"),
                "traffic_stale": traffic.get("lib_sha16") != lib_sha}
        for k, v in kernels.items():
            t = traffic["kernels"].get(k, {}).get("traffic_bytes_per_launch")
            if t:
                v["traffic"] = t
                v.update(tsrc)
                # the PMC-measured HBM bytes over the same kernel-only duration: the fraction of
                # the HBM peak the kernel actually moves (beside the byte model's "frac")
                v["traffic_gbs"] = t / (v["ms"] * 1e-3) / 1e9
                v["traffic_frac"] = v["traffic_gbs"] / HBM_PEAK_GBS
    if "k_solve" in kernels:
        kernels["k_solve"]["bound"] = (
            "latency: iterates on LDS-resident correspondences (one work-group per pair); per "
            "GN iteration one evaluation (block reduction of 28 f64 terms, 256 threads) and the "
            "serial 6x6 solve -- 'frac' is SURVEY 8(d)'s 36 B x C x evaluations model, "
            "'traffic_frac' the PMC-measured HBM bytes over the same duration")
    line["lib_sha16"] = lib_sha
    mk_name = "k_mask_pose_f64" if args.f64_inputs else "k_mask_pose"
    mk = kernels.get(mk_name)
    if mk and "gbs" in mk:
        line["roofline"] = {"bound": "hbm", "achieved": mk["gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": mk["frac"], "traffic": mk.get("traffic"),
                            "kernel": mk_name,
                            "duration": "kernel-only (one-stream kernel pass, HIP events)",
                            **({k: v for k, v in tsrc.items()} if tsrc and mk.get("traffic") else {})}
        f64 = None if args.edges else _load_profile(F64_JSON, B, N, args.mask_before_features, args.layout)
        flops = f64 and f64.get("f64_flops_per_launch")
        if flops:
            tf = flops / (mk["ms"] * 1e-3) / 1e12
            line["roofline_f64"] = {"bound": "valu_f64", "achieved": tf, "peak": F64_PEAK_TFLOPS,
                                    "unit": "TFLOP/s", "frac": tf / F64_PEAK_TFLOPS,
                                    "kernel": "k_mask_pose", "flops_source": os.path.basename(F64_JSON)}
    # the step as a whole: every kernel of the front-end runs once per step, so the step's
    # algorithmic bytes (and PMC bytes) over the measured overlapped step time -- how much of HBM
    # the pipeline moves, beside the single-kernel roofline above (whose kernel-only duration
    # includes its launch's slowest frame)
    step_bytes = sum(v["bytes"] for v in kernels.values() if v.get("bytes"))
    if step_bytes and not args.serial:
        st = elapsed / args.steps
        ach = step_bytes / st / 1e9
        line["roofline_step"] = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": ach / HBM_PEAK_GBS, "bytes_per_step": step_bytes,
                                 "kernels": sorted(k for k, v in kernels.items() if v.get("bytes"))}
        tb = sum(v["traffic"] for v in kernels.values() if v.get("traffic"))
        if tb:
            line["roofline_step"].update(traffic_per_step=tb, traffic_frac=tb / st / 1e9 / HBM_PEAK_GBS)
    curv_k = ("k_feat_wave_run",) if args.layout == "carla" else ("k_feat_wave_reg", "k_feat_chunk_reg", "k_feat_chunk", "k_bin_curv")
    ns = {k: kernels[k]["frac"] for k in (*curv_k, "k_solve") if k in kernels and "frac" in kernels[k]}
    if ns:
        line["north_star_kernels_hbm_frac"] = ns
        meas = {k: kernels[k]["traffic_frac"] for k in ns if "traffic_frac" in kernels[k]}
        if meas:
            line["north_star_kernels_hbm_frac_pmc"] = meas
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
