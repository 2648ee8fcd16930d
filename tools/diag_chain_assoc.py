"""configs[2] chain diagnostic: 33 consecutive frames of ONE sequence (the bench's BatchScanner
data), mask before features, then the 32 chained registrations one by one with HIP events around
each; with the -DSSF_ASSOC_COUNT build (SSF_LIB=.../libssf_frontend_acount.so) nn holds every
query's visited-candidate count: per pair the association time next to the walk statistics
(mean, p99, max, per-wave max) that set it."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ssf-slam_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import ssf
    from ssf import synth
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    count = "acount" in os.path.basename(os.environ.get("SSF_LIB", ""))
    stamps = "sstamp" in os.path.basename(os.environ.get("SSF_LIB", ""))
    dev = torch.device("cuda", 0)
    N = 64 * 1875
    sc = synth.BatchScanner([0], K + 1, n_rows=64, n_az=1875, device=dev)
    pos = torch.empty(((K + 1) * N, 3), dtype=torch.float32, device=dev)
    flow = torch.empty_like(pos)
    for k in range(K + 1):
        sc.frame(k, pos[k * N:(k + 1) * N], flow[k * N:(k + 1) * N])
    off, h_off = ssf.frame_offsets([N] * (K + 1), dev)
    fe = ssf.Frontend(64, device=0, solver="gn", max_iter=10)
    fe.reserve(K + 1, N)
    fe.seed(20240000)
    out, bg = fe.mask_pose(pos, flow, off, h_off, mode="gmm", want_mask=True)
    pb = fe.extract_planes_batch(pos, off, h_off, max_points=N, keep=bg)
    table = fe.plane_table(pb)
    torch.cuda.synchronize()
    cnt = pb.count.cpu().numpy()
    print("plane points per frame: min %d max %d bound %d" % (cnt.min(), cnt.max(), pb.max_points))
    rel = ssf.identity_poses(1, dev)

    def view(a):
        return ssf.PlaneBatch(pb.xyzi, pb.count[a:a + 1], pb.off[a:a + 2], pb.h_off[a:a + 2], pb.max_points)

    for rep in range(2):
        rel.copy_(ssf.identity_poses(1, dev))
        for k in range(K):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            res = fe.register(view(k), table, view(k + 1), rel, want_nn=count or stamps)
            e1.record()
            torch.cuda.synchronize()
            if rep == 0:
                continue
            line = "pair %2d: %4d queries  %.1f us  ncorr %d  t %s" % (
                k, cnt[k + 1], e0.elapsed_time(e1) * 1e3, int(res["ncorr"][0]),
                np.round(rel[0, 4:].cpu().numpy(), 3))
            if count:
                o = int(pb.h_off[k + 1])
                v = res["nn"][o:o + cnt[k + 1]].cpu().numpy().astype(np.int64)
                nd = int((v < 0).sum())
                v = v[v >= 0]
                ns = v >> 16
                v = v & 0xffff
                wm = [v[i:i + 64].max() for i in range(0, len(v), 64)]
                line += "  visits mean %.1f p99 %.0f max %d  wave-max mean %.1f  >500: %d" % (
                    v.mean(), np.percentile(v, 99), v.max(), np.mean(wm), int((v > 500).sum()))
                line += "  deferred %d" % nd
                line += "  strip searches mean %.1f p99 %.0f max %d wave-max mean %.1f" % (
                    ns.mean(), np.percentile(ns, 99), ns.max(), np.mean([ns[i:i + 64].max() for i in range(0, len(ns), 64)]))
            if stamps:
                o = int(pb.h_off[k + 1])
                ny = (cnt[k + 1] + 1023) // 1024
                st = np.stack([res["nn"][o + 1024 * y:o + 1024 * y + 8].cpu().numpy() for y in range(ny)])
                r0 = st[:, 4].min()
                line += "\n   " + "  ".join(
                    "wg%d: stage %.1f lanes %.1f total %.1f us, %d deferred, start +%.1f" % (
                        y, st[y, 0] / 100, st[y, 2] / 100, st[y, 1] / 100, st[y, 3], (st[y, 4] - r0) / 100)
                    for y in range(ny))
            print(line, flush=True)


if __name__ == "__main__":
    main()
