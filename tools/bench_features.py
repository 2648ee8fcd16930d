"""Kernel-only times of the frameFeature chain (+ plane table, association, solve) on B synthetic
frames, through one Frontend context with ssf_profile_enable, on one stream.  Compare library
variants by running it under different SSF_LIB (build.py build_variant).

    python tools/bench_features.py [--batch 256] [--n-az 1875] [--reps 5] [--distinct 16]
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
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--n-az", type=int, default=1875)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--distinct", type=int, default=16)
    ap.add_argument("--chain", action="store_true", help="also plane table + registration")
    ap.add_argument("--layout", default="azimuth", choices=["azimuth", "carla"])
    ap.add_argument("--solver", default="gn", choices=["gn", "ceres_lm"])
    ap.add_argument("--tag", default=os.environ.get("SSF_LIB", "default"))
    ap.add_argument("--dump", default=None, help="with --chain: write the last plane table (normals, validity) "
                    "and registration poses to this .npz")
    ap.add_argument("--stamps", action="store_true",
                    help="diagnostic library (-DSSF_SOLVE_STAMPS): print k_solve phase cycles")
    a = ap.parse_args()
    import ssf
    from ssf import synth
    dev = torch.device("cuda", 0)
    B, N = a.batch, 64 * a.n_az
    pos = [torch.empty((B * N, 3), dtype=torch.float32, device=dev) for _ in range(2)]
    for s in range(a.distinct):
        sc = synth.Scene(s)
        for k in range(2):
            f = synth.scan(s, k, n_az=a.n_az, device=dev, scene=sc, layout=a.layout)
            for b in range(s, B, a.distinct):
                pos[k][b * N:(b + 1) * N].copy_(f["pos1"])
    off, h_off = ssf.frame_offsets([N] * B, dev)
    fe = ssf.Frontend(64, device=0, solver=a.solver, max_iter=10 if a.solver == "gn" else 8)
    fe.reserve(B, N)
    rel = ssf.identity_poses(B, dev)
    for r in range(a.reps + 1):
        if r == 1:
            torch.cuda.synchronize()
            fe.kernel_times()
            fe.profile(True)
        pb0 = fe.extract_planes_batch(pos[0], off, h_off, max_points=N)
        if a.chain:
            t0 = fe.plane_table(pb0)
            pb1 = fe.extract_planes_batch(pos[1], off, h_off, max_points=N)
            res = fe.register(pb0, t0, pb1, rel, want_log=a.stamps)
    torch.cuda.synchronize()
    if a.stamps:
        lg = res["log"][:, -1, 7:10].cpu()
        print(json.dumps({"solve_stamps_cycles": {"compact": float(lg[:, 0].mean()),
                                                  "first_eval": float(lg[:, 1].mean()),
                                                  "iterations": float(lg[:, 2].mean())}}))
    t = fe.kernel_times()
    if a.dump and a.chain:
        import numpy as np
        np.savez(a.dump, normal=t0[0].cpu().numpy(), valid=t0[1].cpu().numpy(), pose=res["pose_rel"].cpu().numpy())
    print(json.dumps({"tag": a.tag, "batch": B, "points": N, "layout": a.layout,
                      "kernel_ms": {k: round(ms / n, 4) for k, (n, ms) in sorted(t.items())}}))


if __name__ == "__main__":
    main()
