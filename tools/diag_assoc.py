"""Association + solve timing on B frame pairs (bench frames), for rocprofv3 --kernel-trace.
Diagnostic only: python tools/diag_assoc.py [B]."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ssf-slam_amd"), REPO]
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
    for rep in range(3):
        pose = ssf.identity_poses(B, dev)
        fe.register(pb[0], table, pb[1], pose)
    torch.cuda.synchronize()
    tb = fe.plane_table(pb[0], brute_force=True)
    pose = ssf.identity_poses(B, dev)
    fe.register(pb[0], tb, pb[1], pose)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
