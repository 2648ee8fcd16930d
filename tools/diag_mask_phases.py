"""Per-phase cycle shares of k_mask_pose from the diagnostic build (SSF_LIB=.../libssf_frontend_diag.so).
Read the SHARES, not the absolute time (stamps perturb the kernel)."""
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
    k0 = int(sys.argv[2]) if len(sys.argv) > 2 else 0        # first frame index of the sequences
    dev = torch.device("cuda", 0)
    fr = [synth.scan(s, k0 + 7 * s, device=dev) for s in range(8)]
    pts = torch.cat([fr[b % 8]["pos1"] for b in range(B)]).contiguous()
    flow = torch.cat([fr[b % 8]["flow"] for b in range(B)]).contiguous()
    N = fr[0]["pos1"].shape[0]
    off, h_off = ssf.frame_offsets([N] * B, dev)
    fe = ssf.Frontend(64, device=0)
    fe.seed(1)
    fe.mask_pose(pts, flow, off, h_off)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out, _ = fe.mask_pose(pts, flow, off, h_off)
    e1.record()
    torch.cuda.synchronize()
    wall_ms = e0.elapsed_time(e1)
    o = out.cpu().numpy()
    st = o[:, 26:32]
    names = ["pass0", "kmeans++", "lloyd", "gmm_init", "em", "final+mask"]
    d = np.diff(np.concatenate([np.zeros((B, 1)), st], 1), axis=1)
    tot = st[:, 5].mean()
    print(f"B={B} mean cycles/frame {tot:.3e}; km_iter {o[:, 19].mean():.1f} em_iter {o[:, 20].mean():.1f} "
          f"passes {o[:, 25].mean():.1f}")
    print(f"  lloyd skip passes: {o[:, 22].mean():.3e} cycles each, {100 * o[:, 23].mean():.2f} % of points relabelled;"
          f" full pass 1 {o[:, 17].mean():.3e}, record-writing full pass {o[:, 21].mean():.3e} cycles")
    slow = int(np.argmax(st[:, 5]))
    print(f"  frame cycles min {st[:, 5].min():.3e} max {st[:, 5].max():.3e} (slowest: km_iter "
          f"{o[slow, 19]:.0f} em_iter {o[slow, 20]:.0f}); kernel wall {wall_ms:.3f} ms -> "
          f"{st[:, 5].max() / wall_ms / 1e6:.2f} G stamp-cycles/s over the slowest frame")
    print(f"  EM pass split (diag slots 0-2): points + block sum {o[:, 0].mean():.3e}, exchange "
          f"{o[:, 1].mean():.3e}, M-step {o[:, 2].mean():.3e} cycles")
    for k, nme in enumerate(names):
        per = ""
        if nme == "lloyd":
            per = f"  per pass {d[:, k].mean() / o[:, 19].mean():.3e}"
        if nme == "em":
            per = f"  per pass {d[:, k].mean() / o[:, 20].mean():.3e}"
        print(f"  {nme:12s} {d[:, k].mean():.3e} cyc  {100 * d[:, k].mean() / tot:5.1f} %{per}")


if __name__ == "__main__":
    main()
