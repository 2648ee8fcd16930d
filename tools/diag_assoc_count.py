"""Phase-1 walk lengths of k_associate_lds per query (diagnostic build -DSSF_ASSOC_COUNT, loaded
through SSF_LIB): mean / percentiles per query, and the per-wave maximum (64 consecutive queries)
that sets a wave's time."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ssf-slam_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import ssf
    from ssf import synth
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    dev = torch.device("cuda", 0)
    fr = [[synth.scan(s, k, device=dev, scene=synth.Scene(s))["pos1"] for k in range(2)] for s in range(8)]
    N = fr[0][0].shape[0]
    off, h_off = ssf.frame_offsets([N] * B, dev)
    fe = ssf.Frontend(64, device=0, solver="gn", max_iter=10)
    pb = [fe.extract_planes_batch(torch.cat([fr[b % 8][k] for b in range(B)]).contiguous(), off, h_off,
                                  max_points=N) for k in range(2)]
    table = fe.plane_table(pb[0])
    ctab = fe.plane_table(pb[1])                      # the curr frames' own x order
    pose = ssf.identity_poses(B, dev)
    pose[:, 4] = 1.0                                       # ~ the synthetic ego motion
    res = fe.register(pb[0], table, pb[1], pose.clone(), want_nn=True)
    torch.cuda.synchronize()
    nn = res["nn"].cpu().numpy()
    cnt = pb[1].count.cpu().numpy()
    si = ctab[3].cpu().numpy()
    curr = pb[1].xyzi.cpu().numpy()
    vis, wmax, wmean, p2 = [], [], [], 0
    xmax, xmean, ymax, ymean = [], [], [], []
    for p in range(B):
        o = int(h_off[p])
        v = nn[o:o + cnt[p]].astype(np.int64)
        p2 += int((v < 0).sum())
        v = np.where(v < 0, -1 - v, v)
        vis.append(v)
        for w0 in range(0, len(v), 64):
            wmax.append(v[w0:w0 + 64].max()); wmean.append(v[w0:w0 + 64].mean())
        vx = v[si[o:o + cnt[p]]]                      # the same walks, lanes in x order
        for w0 in range(0, len(vx), 64):
            xmax.append(vx[w0:w0 + 64].max()); xmean.append(vx[w0:w0 + 64].mean())
        vy = v[np.argsort(v, kind="stable")]          # ideal: lanes grouped by walk length
        for w0 in range(0, len(vy), 64):
            ymax.append(vy[w0:w0 + 64].max()); ymean.append(vy[w0:w0 + 64].mean())
    a = np.concatenate(vis)
    print(f"queries {len(a)}: visited mean {a.mean():.1f} p50 {np.percentile(a, 50):.0f} "
          f"p90 {np.percentile(a, 90):.0f} p99 {np.percentile(a, 99):.0f} max {a.max()} | "
          f"phase 2 {p2} ({100.0 * p2 / len(a):.1f} %)")
    wmax, wmean = np.array(wmax), np.array(wmean)
    print(f"waves {len(wmax)}: per-wave max mean {wmax.mean():.1f} (x{wmax.mean() / a.mean():.2f} the mean "
          f"query), lane efficiency {wmean.sum() / wmax.sum():.3f}")
    print(f"lanes in curr x order: lane efficiency {np.sum(xmean) / np.sum(xmax):.3f}; "
          f"sorted by walk length (bound): {np.sum(ymean) / np.sum(ymax):.3f}")


if __name__ == "__main__":
    main()
