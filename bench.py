"""Benchmark: LiDAR front-end frames/sec (mask + feature + GN) on synthetic 64-beam 120k-pt scans.

One step = one new frame for each of B sequences in flight on this GPU, through the whole hot
path (BASELINE.json north_star):
  * scene-flow dynamic-point mask: GaussianMixture(2) fit + Kabsch pose + quaternion
    (PointCloudOdometry_noSeg.py:97-125)                       -> k_mask_pose         [stream A]
  * frameFeature: ring binning, curvature, planar selection (frameFeature.cpp:45-123)
                                                               -> k_bin_* / k_curv_select / k_compact
  * plane table of the new frame (it is the next step's last frame) + registration of the pair
    (previous frame, new frame): association + 10 Gauss-Newton iterations + pose accumulation
    (lidarOdometry_onlyPC.cpp:147-252, :87-90)                 -> k_plane_table / k_associate / k_solve
                                                                                      [stream B]
  * N > 1: one RCCL all_gather of the step's per-frame 6-DoF poses (weak scaling: every rank
    owns B sequences, no other data-path collective).
Inputs are resident in HBM before the timed region.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(REPO, "ssf-slam_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# HBM bytes per k_mask_pose launch measured with rocprofv3 PMC passes on this bench command
# (tools/pmc_traffic.py: FETCH_SIZE x2 + WRITE_SIZE); used when its workload config matches.
TRAFFIC_JSON = os.path.join(REPO, "profiles", "r01_k_mask_pose_traffic.json")


def mask_traffic(B, N):
    try:
        with open(TRAFFIC_JSON) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    cfg = t.get("config", {})
    if cfg.get("sequences_per_gpu") != B or cfg.get("points_per_frame") != N:
        return None
    return t.get("traffic_bytes_per_launch")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="sequences in flight per GPU")
    ap.add_argument("--n-az", type=int, default=1875, help="azimuth steps (64 x 1875 = 120k pts)")
    ap.add_argument("--rows", type=int, default=64)
    ap.add_argument("--solver", default="gn", choices=["gn", "ceres_lm"])
    ap.add_argument("--iters", type=int, default=None)
    ap.add_argument("--distinct", type=int, default=8, help="distinct synthetic sequences (tiled)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="CPU baseline sample: run the oracle for at least this long (bounded)")
    ap.add_argument("--serial", action="store_true", help="one stream (per-kernel timing without overlap)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N>1 rehearsal on a one-GPU box: every rank on cuda:0, gloo collectives "
                         "(the printed line is marked rehearsal; not a scaling measurement)")
    ap.add_argument("--feat-priority", type=int, default=-1,
                    help="HIP stream priority of the features/registration stream (lower = higher)")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="registration on the features stream (default: its own stream and context, so "
                         "features + plane table of step k+1 run ahead of the registration of step k; "
                         "measured 40.7-40.9k -> 43.8-44.2k frames/s, poses bit-identical)")
    ap.add_argument("--dump-poses", default=None,
                    help="save the accumulated poses after the timed steps (.npy; stream-order check)")
    ap.add_argument("--mask-lag", type=int, default=0,
                    help="mask launch k waits for the registration chain of step k-lag (0: no throttle)")
    ap.add_argument("--mask-streams", type=int, default=3,
                    help="mask launches of consecutive steps alternate over this many streams: the "
                         "GMM of a frame depends on no other frame, so a step's slow frames overlap "
                         "the next step's mask instead of idling the other CUs")
    return ap.parse_args()


def make_data(args, dev, n_frames, rank):
    """[n_frames] batches of B frames: pos/flow packed [B*N, 3] f32, resident in HBM."""
    from ssf import synth
    S = max(1, min(args.distinct, args.batch))
    seqs = []
    for s in range(S):
        seq_id = rank * 1000 + s
        sc = synth.Scene(seq_id)
        fr = [synth.scan(seq_id, k, n_rows=args.rows, n_az=args.n_az, device=dev, scene=sc)
              for k in range(n_frames)]
        seqs.append(fr)
    batches = []
    for k in range(n_frames):
        pos = torch.cat([seqs[b % S][k]["pos1"] for b in range(args.batch)]).contiguous()
        flow = torch.cat([seqs[b % S][k]["flow"] for b in range(args.batch)]).contiguous()
        batches.append((pos, flow))
    del seqs
    return batches


def cpu_baseline(args):
    """The CPU oracle (C restatement of the reference path, single thread) on a bounded sample:
    frames of one synthetic sequence through mask + features + plane table + registration
    (warm-started pairs, frames cycled), timed on this host until >= cpu_seconds have elapsed."""
    from oracle import oracle as O
    from ssf import synth
    O.lib()
    sc = synth.Scene(0)
    n_src = 4
    fr = [synth.scan(0, k, n_rows=args.rows, n_az=args.n_az, scene=sc) for k in range(n_src)]
    fr = [(f["pos1"].numpy(), f["flow"].numpy()) for f in fr]
    prof = O.profile(args.rows)
    mode = O.MODE_GN if args.solver == "gn" else O.MODE_CERES_LM
    iters = args.iters or (10 if args.solver == "gn" else 8)
    last = O.extract_planes(fr[0][0], args.rows)
    q, t = np.array([0, 0, 0, 1.0]), np.zeros(3)
    done = 0
    t0 = time.perf_counter()
    while True:
        p, f = fr[1 + done % (n_src - 1)]
        O.mask_and_pose(p, f, [0.3, 0.6, 0.9])
        curr = O.extract_planes(p, args.rows)
        q, t, _, _ = O.register_pair(last, curr, prof.plane_max, mode=mode, max_iter=iters, q_init=q, t_init=t)
        last = curr
        done += 1
        el = time.perf_counter() - t0
        if (el >= args.cpu_seconds and done >= 2) or el > 30.0:
            break
    return dict(value=done / el, unit="frames/s", cores=1, kind="port",
                sample=f"{done} frames of {args.rows}-beam {args.rows * args.n_az}-pt synthetic scans "
                       f"(mask+features+plane table+{args.solver} x{iters}) through oracle/ssf_oracle.c, "
                       f"1 thread, {el:.2f} s")


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.warmup < 1:
        args.warmup = 1  # the first frame of a sequence has no last frame to register against
    if args.rehearse_one_gpu:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    import ssf
    from ssf import dist as sd
    iters = args.iters or (10 if args.solver == "gn" else 8)
    B, N = args.batch, args.rows * args.n_az
    n_frames = args.warmup + args.steps + 1
    batches = make_data(args, dev, n_frames, rank)
    off, h_off = ssf.frame_offsets([N] * B, dev)
    fe_mask = ssf.Frontend(args.rows, device=local)
    fe_feat = ssf.Frontend(args.rows, device=local, solver=args.solver, max_iter=iters)
    fe_mask.reserve(B, N)
    fe_feat.reserve(B, N)
    fe_mask.seed(20240000 + rank)
    n_ms = 1 if args.serial else max(1, args.mask_streams)
    s_masks = [torch.cuda.Stream(dev) for _ in range(n_ms)]
    # the registration chain is serial across steps: its stream gets the higher priority so the
    # mask launches (independent frames) fill the CUs it leaves free
    s_feat = s_masks[0] if args.serial else torch.cuda.Stream(dev, priority=args.feat_priority)
    # registration on its own stream and context: features + plane table of step k + 1 do not
    # wait for the registration of step k (it only needs the plane table of its two frames)
    s_reg = s_feat if args.serial or not args.pipeline else torch.cuda.Stream(dev, priority=args.feat_priority)
    fe_reg = fe_feat if s_reg is s_feat else ssf.Frontend(args.rows, device=local, solver=args.solver,
                                                          max_iter=iters)
    if fe_reg is not fe_feat:
        fe_reg.reserve(B, N)
    # per-step outputs (double-buffered plane clouds: last <- curr)
    pose_rel = ssf.identity_poses(B, dev)
    pose_abs = ssf.identity_poses(B, dev)
    mask_out = [None] * n_frames
    gathered = []
    ev = {k: [] for k in ("mask", "feat", "table", "reg")}
    state = {"last": None, "last_table": None}
    chain_done = [None] * n_frames

    def step(k, timing):
        pos, flow = batches[k]
        s_mask = s_masks[k % n_ms]
        # optional throttle (off by default): mask k waits for the registration chain of step
        # k-lag.  Measured: 33.2-33.9 k frames/s with lag 1-3 against 39.5 k without -- the
        # unthrottled masks overlap each other's straggler tails, and the chain catches up
        if not args.serial and args.mask_lag > 0 and k - args.mask_lag >= 0:
            s_mask.wait_event(chain_done[k - args.mask_lag])
        with torch.cuda.stream(s_mask):
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s_mask)
            out, bg = fe_mask.mask_pose(pos, flow, off, h_off, mode="gmm", want_mask=True)
            e1.record(s_mask)
            mask_out[k] = out
        with torch.cuda.stream(s_feat):
            es = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            es[0].record(s_feat)
            pb = fe_feat.extract_planes_batch(pos, off, h_off, max_points=N)
            es[1].record(s_feat)
            table = fe_feat.plane_table(pb)
            es[2].record(s_feat)
        if s_reg is not s_feat:
            s_reg.wait_event(es[2])
            # the plane batch and its table are read on s_reg in this step and the next: keep
            # the caching allocator from handing their blocks to s_feat until s_reg is done
            for t in (pb.xyzi, pb.count, *[x for x in table if isinstance(x, torch.Tensor)]):
                t.record_stream(s_reg)
        with torch.cuda.stream(s_reg):
            if state["last"] is not None:
                fe_reg.register(state["last"], state["last_table"], pb, pose_rel, pose_abs)
            es[3].record(s_reg)
            chain_done[k] = torch.cuda.Event()
            chain_done[k].record(s_reg)
        state["last"], state["last_table"] = pb, table
        if world > 1:   # the one exchange step: per-frame 6-DoF poses of every rank (RCCL)
            cur = torch.cuda.current_stream(dev)
            cur.wait_stream(s_mask)
            cur.wait_stream(s_feat)
            cur.wait_stream(s_reg)
            gathered.append(sd.gather_poses(sd.pose_record(pose_abs, mask_out[k])))
        if timing:
            ev["mask"].append((e0, e1)); ev["feat"].append((es[0], es[1]))
            ev["table"].append((es[1], es[2])); ev["reg"].append((es[2], es[3]))

    for k in range(args.warmup):
        step(k, False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        step(k, True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if args.dump_poses and rank == 0:
        np.save(args.dump_poses, pose_abs.cpu().numpy())
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if args.rehearse_one_gpu else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- per-kernel timing (HIP events on the launching streams) + algorithmic bytes
    def avg_ms(pairs):
        return float(np.mean([a.elapsed_time(b) for a, b in pairs]))

    mask_ms = avg_ms(ev["mask"])
    feat_ms = avg_ms(ev["feat"])
    table_ms = avg_ms(ev["table"])
    reg_ms = avg_ms(ev["reg"])
    passes = torch.stack([mask_out[k][:, 25] for k in range(args.warmup, args.warmup + args.steps)])
    status = torch.stack([mask_out[k][:, 16] for k in range(args.warmup, args.warmup + args.steps)])
    mean_passes = float(passes.mean())
    # k_mask_pose: out[25] counts its algorithmic bytes in units of one [flow, xyz] float32
    # stream (24 B/pt; Lloyd skip passes count their record/queue bytes); + 1 B/pt mask write
    mask_bytes = B * N * (24.0 * mean_passes + 1.0)
    # frameFeature chain: bin_count 12 R + 1 W, bin_scatter 13 R + 16 W, curv_select 16 R + 4 W(sel)
    feat_bytes = B * N * (12 + 1 + 13 + 16 + 16) * 1.0
    kernels = {
        # gbs: per launch (launches of consecutive steps overlap on two streams, so a launch's
        # duration includes time shared with the next one); aggregate_gbs: all mask bytes of the
        # timed steps over the timed wall time
        "k_mask_pose": dict(ms=mask_ms, bytes=mask_bytes, gbs=mask_bytes / mask_ms / 1e6,
                            aggregate_gbs=mask_bytes * args.steps / elapsed / 1e9,
                            passes_per_frame=mean_passes, streams=n_ms),
        "features(5 kernels)": dict(ms=feat_ms, bytes=feat_bytes, gbs=feat_bytes / feat_ms / 1e6),
        "plane_table": dict(ms=table_ms),
        "register(assoc+solve)": dict(ms=reg_ms),
    }
    dom = max(kernels, key=lambda k: kernels[k]["ms"])
    total_frames = B * args.steps * world
    value = total_frames / elapsed
    line = {
        "metric": "LiDAR front-end frames/sec (mask+feature+GN), 64-beam 120k pts, 1/2/4/8 GPUs",
        "value": value, "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32 features / f64 mask+solve",
        "data": "synthetic (seeded ray-cast 64-beam scans, ssf/synth.py)",
        "config": {"workload": f"{B} sequences in flight per GPU x {args.rows}-beam {N}-pt scans; "
                               f"mask(GMM+Kabsch) + features + plane table + {args.solver} x{iters}",
                   "sequences_per_gpu": B, "points_per_frame": N, "solver": args.solver,
                   "iters": iters, "parallelism": f"sequence-sharded x{world}",
                   **({"rehearsal": "all ranks on one GPU, gloo"} if args.rehearse_one_gpu else {})},
        "roofline": None, "cpu_baseline": None, "kernels": kernels,
        "mask_status_nonzero": int((status != 0).sum()),
    }
    if "k_mask_pose" == dom:
        achieved = mask_bytes / (mask_ms * 1e-3) / 1e9
        line["roofline"] = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": achieved / HBM_PEAK_GBS, "traffic": mask_traffic(B, N),
                            "kernel": "k_mask_pose"}
    else:
        k = kernels[dom]
        b = k.get("bytes")
        if b:
            achieved = b / (k["ms"] * 1e-3) / 1e9
            line["roofline"] = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                                "kernel": dom}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
