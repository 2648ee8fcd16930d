"""Time the TFlow point-set operators at the network's first
set-abstraction shape (scripts/ActiveSceneFlow/TFlowV3_Occlussion.py:69-70: 8192 input points,
sa1 npoint 2048, nsample 16) on one MI355X, with the single-thread CPU oracle beside it.

    python tools/bench_pn2.py [--clouds 64] [--reps 10] [--out profiles/r01_pn2_bench.json]

Per op: HIP-event time per launch on torch's current stream (the stream the ops launch on),
algorithmic bytes (inputs read once + outputs written once) and the HBM fraction, or the
distance-evaluation rate for the brute-force searches (VALU-bound).  Synthetic clouds
(seeded normal, 20 m scale); the oracle runs one cloud (scaled to the batch in the report).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ssf-slam_amd"), REPO]

HBM_PEAK = 8000.0  # GB/s, /opt/skills/guides/MI355X_MICROARCH.md


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clouds", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from ssf import pointnet2 as P
    from oracle import oracle as O

    dev = torch.device("cuda", 0)
    B, N, S, K, C, KU = a.clouds, 8192, 2048, 16, 35, 7
    rng = np.random.default_rng(0)
    xyz_h = (rng.standard_normal((B, N, 3)) * 20).astype(np.float32)
    xyz = torch.from_numpy(xyz_h).to(dev)
    feat = torch.randn(B, C, N, device=dev)
    fps = P.furthest_point_sample(xyz, S)
    new_xyz = torch.gather(xyz, 1, fps.long().unsqueeze(-1).expand(-1, -1, 3)).contiguous()
    _, idx = P.knn(K, new_xyz, xyz)
    xyz_c = xyz.permute(0, 2, 1).contiguous()
    sxyz_c = new_xyz.permute(0, 2, 1).contiguous()
    sflow = torch.randn(B, 3, S, device=dev)
    torch.cuda.synchronize()

    res = {}
    ms = timed(lambda: P.furthest_point_sample(xyz, S), a.reps)
    res["furthest_point_sample"] = dict(ms=ms, clouds_per_s=B / ms * 1e3,
                                        dist_evals_per_s=B * N * (S - 1) / ms * 1e3,
                                        bound="latency (one barrier per centroid)")
    ms = timed(lambda: P.knn(K, new_xyz, xyz), a.reps)
    res["knn"] = dict(ms=ms, pairs_per_s=B * S * N / ms * 1e3, bound="VALU (brute force)")
    ms = timed(lambda: P.grouping_operation(feat, idx), a.reps)
    by = B * C * N * 4 + B * S * K * 4 + B * C * S * K * 4   # feature map + indices read once, output written
    res["grouping_operation"] = dict(ms=ms, bytes=by, gbs=by / ms / 1e6,
                                     frac=by / ms / 1e6 / HBM_PEAK, bound="hbm")
    pts32 = torch.randn(B, 32, N, device=dev)
    ms = timed(lambda: P.group_relative(xyz_c, sxyz_c, pts32, idx), a.reps)
    by = B * 35 * N * 4 + B * 3 * S * 4 + B * S * K * 4 * 2 + B * 35 * S * K * 4
    res["group_relative"] = dict(ms=ms, bytes=by, gbs=by / ms / 1e6, frac=by / ms / 1e6 / HBM_PEAK,
                                 bound="hbm", shape=f"sa1: [B, 3+32, {S}, {K}] from {N} points")
    i3 = torch.randint(0, S, (B, N, 3), device=dev, dtype=torch.int32)
    w3 = torch.rand(B, N, 3, device=dev)
    sfeat = torch.randn(B, 64, S, device=dev)
    ms = timed(lambda: P.three_interpolate(sfeat, i3, w3), a.reps)
    by = B * 64 * S * 4 + B * N * 3 * 8 + B * 64 * N * 4
    res["three_interpolate"] = dict(ms=ms, bytes=by, gbs=by / ms / 1e6, frac=by / ms / 1e6 / HBM_PEAK,
                                    bound="hbm", shape=f"C=64, {S} -> {N}")
    ms = timed(lambda: P.upsample_flow(xyz_c, sxyz_c, sflow, k=KU), a.reps)
    res["upsample_flow"] = dict(ms=ms, pairs_per_s=B * N * S / ms * 1e3,
                                bound="VALU (brute force over the LDS-staged sparse cloud)")

    # CPU oracle on one cloud (single thread), same shapes
    t = time.perf_counter(); fo = O.pn2_fps(xyz_h[:1], S); t_fps = time.perf_counter() - t
    nx = np.take_along_axis(xyz_h[:1], fo[..., None].astype(np.int64), axis=1)
    t = time.perf_counter(); O.pn2_knn(K, nx, xyz_h[:1]); t_knn = time.perf_counter() - t
    assert np.array_equal(fo, fps[:1].cpu().numpy()), "GPU FPS differs from the oracle"
    line = dict(workload=f"{B} clouds x {N} pts: FPS -> {S}, knn k={K} ({S} queries), grouping "
                         f"C={C} K={K}, UpsampleFlow k={KU} from {S}",
                ops=res,
                cpu_oracle=dict(fps_s_per_cloud=t_fps, knn_s_per_cloud=t_knn, cores=1, kind="port"),
                speedup_vs_oracle=dict(fps=t_fps * B / (res["furthest_point_sample"]["ms"] / 1e3),
                                       knn=t_knn * B / (res["knn"]["ms"] / 1e3)))
    print(json.dumps(line))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(line, f, indent=1)


if __name__ == "__main__":
    main()
