"""BatchScanner (GPU ray cast, libssf_synth.so) vs synth.scan (torch) on the same (seq, frame):
per-sequence position / flow differences (only the noise draws differ, so |dpos| ~ range noise
except at object silhouettes), plus the registration of frame 0 -> 1 of each sequence with both
data sets (GN poses vs the ground-truth relative pose)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "ssf-slam_amd"), REPO):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import ssf
    from ssf import synth
    dev = torch.device("cuda", 0)
    seqs = [int(s) for s in sys.argv[1].split(",")] if len(sys.argv) > 1 else list(range(0, 256, 17))
    N = 64 * 1875
    sc = synth.BatchScanner(seqs, 4, device=dev)
    frames = []
    for k in range(3):
        pos = torch.empty((len(seqs) * N, 3), dtype=torch.float32, device=dev)
        flow = torch.empty_like(pos)
        sc.frame(k, pos, flow)
        frames.append((pos, flow))
    torch.cuda.synchronize()
    fe = ssf.Frontend(64, device=0, solver="gn", max_iter=10)
    B = len(seqs)
    off, h_off = ssf.frame_offsets([N] * B, dev)
    out = {}
    ref_pos = [torch.cat([synth.scan(s, k, device=dev)["pos1"] for s in seqs]) for k in range(2)]
    for name, P in (("batch", [frames[0][0], frames[1][0]]), ("torch", ref_pos)):
        pb0 = fe.extract_planes_batch(P[0], off, h_off, max_points=N)
        tb = fe.plane_table(pb0)
        pb1 = fe.extract_planes_batch(P[1], off, h_off, max_points=N)
        rel = ssf.identity_poses(B, dev)
        fe.register(pb0, tb, pb1, rel)
        torch.cuda.synchronize()
        out[name] = dict(planes=pb0.count.cpu().tolist(), t=rel[:, 4:].cpu().numpy().round(4).tolist())
    dpos = (frames[0][0] - ref_pos[0]).abs().view(B, N, 3).amax(2)
    res = {"seqs": seqs, "dpos_median": dpos.median(1).values.cpu().tolist(),
           "dpos_frac_gt_0.2m": (dpos > 0.2).float().mean(1).cpu().tolist(),
           "gt_t": [list(synth.relative_pose(s, 0, 1)[1]) for s in seqs], **out}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
