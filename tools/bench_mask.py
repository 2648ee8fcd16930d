"""Kernel-only time of k_mask_pose (GMM fit + Kabsch) for B frames at several frame splits
(ssf_set_mask_split), one stream, HIP events via ssf_profile_enable; also checks that every
split gives the same labels / iteration counts as split 1 (summation order aside).

    python tools/bench_mask.py --batch 32 --splits 1,2,4,8 [--reps 3] [--distinct 32]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "ssf-slam_amd"), REPO):
    sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--n-az", type=int, default=1875)
    ap.add_argument("--splits", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--distinct", type=int, default=32)
    ap.add_argument("--dump", default=None, help="write the first split's outputs (out, mask) to this .npz")
    a = ap.parse_args()
    import ssf
    from ssf import synth
    dev = torch.device("cuda", 0)
    B, N = a.batch, 64 * a.n_az
    pos = torch.empty((B * N, 3), dtype=torch.float32, device=dev)
    flow = torch.empty_like(pos)
    for s in range(min(a.distinct, B)):
        f = synth.scan(s, 1, n_az=a.n_az, device=dev, scene=synth.Scene(s))
        for b in range(s, B, min(a.distinct, B)):
            pos[b * N:(b + 1) * N].copy_(f["pos1"])
            flow[b * N:(b + 1) * N].copy_(f["flow"])
    off, h_off = ssf.frame_offsets([N] * B, dev)
    draws = torch.rand((B, 3), dtype=torch.float64, generator=torch.Generator().manual_seed(5)).numpy()
    fe = ssf.Frontend(64, device=0)
    fe.reserve(B, N)
    ref = None
    res = {}
    for G in [int(x) for x in a.splits.split(",")]:
        fe.mask_split(G)
        out, bg = fe.mask_pose(pos, flow, off, h_off, draws=draws)          # warm-up
        torch.cuda.synchronize()
        fe.kernel_times()
        fe.profile(True)
        for _ in range(a.reps):
            out, bg = fe.mask_pose(pos, flow, off, h_off, draws=draws)
        torch.cuda.synchronize()
        fe.profile(False)
        n, ms = fe.kernel_times()["k_mask_pose"]
        o = out.cpu()
        st = o[:, 16]
        row = dict(ms=round(ms / n, 3), status_nonzero=int((st != 0).sum()),
                   km_iter=float(o[:, 19].mean()), em_iter=float(o[:, 20].mean()))
        if ref is None:
            ref = (o.clone(), bg.cpu().clone())
            if a.dump:
                import numpy as np
                np.savez(a.dump, out=o.numpy(), bg=bg.cpu().numpy())
        else:
            row["labels_equal_split1"] = float((bg.cpu() == ref[1]).float().mean())
            row["iters_equal_split1"] = bool(torch.equal(o[:, 19:21], ref[0][:, 19:21]))
            row["max_dt_vs_split1"] = float((o[:, 0:3] - ref[0][:, 0:3]).abs().max())
        res[G] = row
        print(json.dumps({"batch": B, "split": G, **row}), flush=True)


if __name__ == "__main__":
    main()
