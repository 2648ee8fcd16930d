"""Mask-only throughput: k_mask_pose launches of B frames round-robin over S streams (one
Frontend context per stream), as bench.py keeps its mask launches in flight, with nothing else on
the GPU -- the ceiling the full pipeline's frames/s would reach if the feature / table /
registration chain cost no CU time.

    python tools/bench_mask_overlap.py [--batch 256] [--streams 1,2,3,4] [--launches 30]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "ssf-slam_amd"), REPO):
    sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--n-az", type=int, default=1875)
    ap.add_argument("--streams", default="1,2,3,4")
    ap.add_argument("--launches", type=int, default=30)
    ap.add_argument("--distinct", type=int, default=32)
    ap.add_argument("--queue", type=int, default=0, help="frame queue of at most this many work-groups "
                    "per launch (ssf_set_mask_schedule; 0: one work-group per frame)")
    a = ap.parse_args()
    import ssf
    from ssf import synth
    dev = torch.device("cuda", 0)
    B, N = a.batch, 64 * a.n_az
    data = []
    for k in range(2):                                        # two batches, alternating
        pos = torch.empty((B * N, 3), dtype=torch.float32, device=dev)
        flow = torch.empty_like(pos)
        for s in range(min(a.distinct, B)):
            f = synth.scan(s + 100 * k, 1, n_az=a.n_az, device=dev, scene=synth.Scene(s + 100 * k))
            for b in range(s, B, min(a.distinct, B)):
                pos[b * N:(b + 1) * N].copy_(f["pos1"])
                flow[b * N:(b + 1) * N].copy_(f["flow"])
        data.append((pos, flow))
    off, h_off = ssf.frame_offsets([N] * B, dev)
    draws = torch.rand((B, 3), dtype=torch.float64, generator=torch.Generator().manual_seed(5)).numpy()
    for S in [int(x) for x in a.streams.split(",")]:
        fes = [ssf.Frontend(64, device=0) for _ in range(S)]
        for fe in fes:
            fe.reserve(B, N)
            if a.queue:
                fe.mask_schedule(None, a.queue)
        streams = [torch.cuda.Stream(dev) for _ in range(S)]

        def run(n):
            for j in range(n):
                with torch.cuda.stream(streams[j % S]):
                    pos, flow = data[j % 2]
                    fes[j % S].mask_pose(pos, flow, off, h_off, draws=draws)
        run(S)                                                # warm-up: every context once
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(a.launches)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"batch": B, "streams": S, "queue": a.queue, "launches": a.launches,
                          "ms_per_launch": round(dt / a.launches * 1e3, 3),
                          "frames_per_s": round(a.launches * B / dt, 1)}), flush=True)
        del fes
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
