"""Dump k_mask_pose outputs (pose records + background mask) of a synthetic batch to .npz, for a
bitwise A/B of two builds (SSF_LIB=... python tools/dump_mask.py B split out.npz; then
tools/cmp_npz.py a.npz b.npz)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ssf-slam_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import ssf
    from ssf import synth
    B, split, path = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    dev = torch.device("cuda", 0)
    fr = [synth.scan(s, 0, device=dev) for s in range(min(B, 8))]
    pts = torch.cat([fr[b % len(fr)]["pos1"] for b in range(B)]).contiguous()
    flow = torch.cat([fr[b % len(fr)]["flow"] for b in range(B)]).contiguous()
    N = fr[0]["pos1"].shape[0]
    off, h_off = ssf.frame_offsets([N] * B, dev)
    fe = ssf.Frontend(64, device=0)
    fe.mask_split(split)
    fe.seed(7)
    out, bg = fe.mask_pose(pts, flow, off, h_off, want_mask=True)
    torch.cuda.synchronize()
    np.savez(path, out=out.cpu().numpy(), bg=bg.cpu().numpy())
    o = out.cpu().numpy()
    print(f"B={B} split={split}: status {np.unique(o[:, 16])}, em_iter mean {o[:, 20].mean():.2f}")


if __name__ == "__main__":
    main()
