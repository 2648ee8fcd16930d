"""Per-frame phase cycles of k_mask_pose (diagnostic build, SSF_LIB=.../libssf_frontend_diag.so)
on the bench's workload: B distinct synthetic sequences (ssf/synth.py), frame k of each.  Writes
an npz with the per-frame stamps and iteration counts, used to size the straggler work (how long
the slowest frames run against the mean, and in which phase).

    SSF_LIB=ssf-slam_amd/ssf/_lib/libssf_frontend_diag.so python tools/diag_mask_frames.py OUT.npz [B]
"""
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
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    dev = torch.device("cuda", 0)
    t0 = time.time()
    fr = [synth.scan(s, 1, device=dev, scene=synth.Scene(s)) for s in range(B)]
    print(f"data {time.time() - t0:.1f} s", flush=True)
    pts = torch.cat([f["pos1"] for f in fr]).contiguous()
    flow = torch.cat([f["flow"] for f in fr]).contiguous()
    off, h_off = ssf.frame_offsets([f["pos1"].shape[0] for f in fr], dev)
    fe = ssf.Frontend(64, device=0)
    fe.seed(1)
    fe.mask_pose(pts, flow, off, h_off)
    torch.cuda.synchronize()
    out, _ = fe.mask_pose(pts, flow, off, h_off)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    np.savez(outp, out=o)
    st = o[:, 26:32]
    print(f"frame cycles mean {st[:, 5].mean():.3e} max {st[:, 5].max():.3e}; km_iter mean "
          f"{o[:, 19].mean():.1f} max {o[:, 19].max():.0f}; em_iter mean {o[:, 20].mean():.1f} max "
          f"{o[:, 20].max():.0f}", flush=True)


if __name__ == "__main__":
    main()
