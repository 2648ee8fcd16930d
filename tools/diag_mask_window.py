"""Per-step cost of the hot path along the synthetic sequences (name the
17-20 % drop of the `--warmup 50` line).  The bench's workload (256 sequences, frame k of each
per step), every stage run SERIALLY on one stream per step with HIP events: mask launch ms and
per-frame EM / Lloyd iteration counts and full-pass equivalents (max vs mean), features, plane
table, registration ms and plane / correspondence counts.

    python tools/diag_mask_window.py OUT.json [n_steps] [B]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ssf-slam_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import ssf
    from ssf import synth
    outp = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 150
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    layout = os.environ.get("LAYOUT", "azimuth")
    dev = torch.device("cuda", 0)
    N = 64 * 1875
    t0 = time.time()
    sc = synth.BatchScanner(list(range(B)), K, n_rows=64, n_az=1875, device=dev, layout=layout)
    pos = torch.empty((B * N, 3), dtype=torch.float32, device=dev)
    flow = torch.empty_like(pos)
    off, h_off = ssf.frame_offsets([N] * B, dev)
    fm = ssf.Frontend(64, device=0)
    ff = ssf.Frontend(64, device=0, solver="gn", max_iter=10)
    fm.reserve(B, N)
    ff.reserve(B, N)
    pose_rel = ssf.identity_poses(B, dev)
    pose_abs = ssf.identity_poses(B, dev)
    ev = lambda: torch.cuda.Event(enable_timing=True)
    rows, last = [], None
    for k in range(K):
        sc.frame(k, pos, flow)
        torch.cuda.synchronize()
        e = [ev() for _ in range(5)]
        e[0].record()
        out, _ = fm.mask_pose(pos, flow, off, h_off, mode="gmm", want_mask=True)
        e[1].record()
        pb = ff.extract_planes_batch(pos, off, h_off, max_points=N)
        e[2].record()
        table = ff.plane_table(pb)
        e[3].record()
        nc = None
        if last is not None:
            res = ff.register(last[0], last[1], pb, pose_rel, pose_abs)
            nc = res["ncorr"]
        e[4].record()
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        km, em, ps = o[:, 19], o[:, 20], o[:, 25]
        r = dict(k=k, mask_ms=e[0].elapsed_time(e[1]), feat_ms=e[1].elapsed_time(e[2]),
                 table_ms=e[2].elapsed_time(e[3]), reg_ms=e[3].elapsed_time(e[4]),
                 km_mean=float(km.mean()), km_max=float(km.max()), em_mean=float(em.mean()),
                 em_max=float(em.max()), passes_mean=float(ps.mean()), passes_max=float(ps.max()),
                 passes_p90=float(np.percentile(ps, 90)), planes_mean=float(pb.count.float().mean()),
                 ncorr_mean=None if nc is None else float(nc.float().mean()))
        rows.append(r)
        # keep a private copy of the plane batch / table for the next pair (pb's buffers are fresh)
        last = (pb, table)
        print(json.dumps({a: (round(b, 3) if isinstance(b, float) else b) for a, b in r.items()}), flush=True)
    json.dump(dict(rows=rows, B=B, layout=layout, gen_s=time.time() - t0), open(outp, "w"), indent=1)


if __name__ == "__main__":
    main()
