"""Phase shares of k_plane_table_sorted (diagnostic build, SSF_LIB=.../libssf_frontend_diag.so)."""
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
    fr = [synth.scan(s, 0, device=dev)["pos1"] for s in range(8)]
    pts = torch.cat([fr[b % 8] for b in range(B)]).contiguous()
    N = fr[0].shape[0]
    off, h_off = ssf.frame_offsets([N] * B, dev)
    fe = ssf.Frontend(64, device=0)
    pb = fe.extract_planes_batch(pts, off, h_off)
    for _ in range(2):
        t = fe.plane_table(pb)
        torch.cuda.synchronize()
    si = t[3].cpu().numpy()
    cnt = pb.count.cpu().numpy()
    st = np.array([si[int(h_off[f]) + cnt[f]: int(h_off[f]) + cnt[f] + 6] for f in range(B)]).astype(np.float64)
    st[:, [0, 1, 3, 4, 5]] *= 16
    for name, red in (("mean", np.mean), ("p90", lambda a: np.percentile(a, 90)), ("max", np.max)):
        print(f"B={B} {name}: m {red(cnt):.0f}; cycles: sort {red(st[:,0]):.3e}  bounded-walks-end "
              f"{red(st[:,1]):.3e} (queue {red(st[:,2]):.0f})  strips-built {red(st[:,4]):.3e}  queue-done {red(st[:,5]):.3e}  end {red(st[:,3]):.3e}")
    f = int(np.argmax(st[:, 3]))
    print(f"slowest frame {f}: m {cnt[f]} sort {st[f,0]:.3e} bounded {st[f,1]:.3e} queue {st[f,2]:.0f} end {st[f,3]:.3e}")


if __name__ == "__main__":
    main()
