"""k_plane_table_sorted alone: ms per B-frame launch (HIP events around each launch, median of
--reps), on frames taken along the sequences (frame 7 s mod 200 of sequence s, as bench.py
--stagger 200), plus a hash of the outputs so two builds can be compared bit for bit.
SSF_LIB picks the build."""
import argparse
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ssf-slam_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--distinct", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import ssf
    from ssf import synth
    dev = torch.device("cuda", 0)
    fr = [synth.scan(s, (7 * s) % 200, device=dev)["pos1"] for s in range(a.distinct)]
    pts = torch.cat([fr[b % a.distinct] for b in range(a.batch)]).contiguous()
    off, h_off = ssf.frame_offsets([f.shape[0] for f in (fr[b % a.distinct] for b in range(a.batch))], dev)
    fe = ssf.Frontend(64, device=0)
    pb = fe.extract_planes_batch(pts, off, h_off)
    t = fe.plane_table(pb)
    torch.cuda.synchronize()
    ms = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t = fe.plane_table(pb, out=t.tensors())
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    h = hashlib.sha256()
    cnt = pb.count.cpu().numpy()
    for x in (t[0], t[1]):
        h.update(x.cpu().numpy().tobytes())
    print(json.dumps({"batch": a.batch, "ms_median": float(np.median(ms)), "ms_min": float(np.min(ms)),
                      "planes_mean": float(cnt.mean()), "valid": int(t[1].sum().item()),
                      "out_sha": h.hexdigest()[:16], "lib": os.path.basename(os.environ.get("SSF_LIB", "default"))}))


if __name__ == "__main__":
    main()
