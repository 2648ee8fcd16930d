"""Per-work-group lifetimes of k_associate_lds (diagnostic build: SSF_LIB=.../libssf_frontend_diag.so)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ssf-slam_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import ssf
    from ssf import synth
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dev = torch.device("cuda", 0)
    fr = [[synth.scan(s, k, device=dev, scene=synth.Scene(s))["pos1"] for k in range(2)] for s in range(8)]
    N = fr[0][0].shape[0]
    off, h_off = ssf.frame_offsets([N] * B, dev)
    fe = ssf.Frontend(64, device=0, solver="gn", max_iter=10)
    pb = [fe.extract_planes_batch(torch.cat([fr[b % 8][k] for b in range(B)]).contiguous(), off, h_off,
                                  max_points=N) for k in range(2)]
    table = fe.plane_table(pb[0])
    for _ in range(2):
        res = fe.register(pb[0], table, pb[1], ssf.identity_poses(B, dev), want_nn=True)
    torch.cuda.synchronize()
    nn = res["nn"].cpu().numpy()
    cnt = pb[1].count.cpu().numpy()
    rows = []
    for p in range(B):
        o = int(h_off[p])
        for wg in range((cnt[p] + 2047) // 2048):
            v = nn[o + 2048 * wg: o + 2048 * wg + 4].astype(np.int64)
            rows.append((p, wg, v[0] << 8, v[1] << 4, v[2] << 4, v[3]))
    a = np.array(rows, dtype=np.float64)
    t0 = a[:, 2].min()
    start = a[:, 2] - t0
    print(f"WGs {len(a)}: phase1 mean {a[:,3].mean():.3e} max {a[:,3].max():.3e} | total mean {a[:,4].mean():.3e} "
          f"max {a[:,4].max():.3e} | start spread max {start.max():.3e} | queued mean {a[:,5].mean():.0f} max {a[:,5].max():.0f}")
    k = int(np.argmax(a[:, 4]))
    print("slowest WG (pair, wg, phase1, total, nq):", int(a[k, 0]), int(a[k, 1]), f"{a[k,3]:.3e}", f"{a[k,4]:.3e}", int(a[k, 5]))
    end = start + a[:, 4]
    print(f"last end {end.max():.3e} cycles after the first start")


if __name__ == "__main__":
    main()
