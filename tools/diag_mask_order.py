"""Does the ORDER of a mask launch's frames matter?  A 256-frame k_mask_pose launch ends with its
slowest frame (up to ~2.7x the mean), and one work-group per frame is dispatched in frame order.
Longest-first (LPT) dispatch shortens that tail.  Frame costs are not known before the fit, but a
sequence's consecutive frames look alike, so the previous step's per-frame cost of the same
sequence (out[:, SSF_POSE_OUT_PASSES]) predicts the next one.

On the bench's workload (B staggered sequences, bench.py make_data): per step, one-stream launch
times of the frames (a) in sequence order, (b) ordered by the previous step's cost, (c) ordered by
their own cost (the bound); then 3-stream overlapped throughput over the steps, (a) vs (b).  The
frames are permuted in memory (a copy), so the kernel is unchanged.

    python tools/diag_mask_order.py OUT.json [steps] [B]
"""
import json
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
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    dev = torch.device("cuda", 0)
    N = 64 * 1875
    sc = synth.BatchScanner(list(range(B)), K, n_rows=64, n_az=1875, device=dev,
                            start=[(7 * b) % 200 for b in range(B)])
    data = []
    for k in range(K):
        pos = torch.empty((B * N, 3), dtype=torch.float32, device=dev)
        flow = torch.empty_like(pos)
        sc.frame(k, pos, flow)
        data.append((pos, flow))
    torch.cuda.synchronize()
    off, h_off = ssf.frame_offsets([N] * B, dev)
    fe = ssf.Frontend(64, device=0)
    fe.reserve(B, N)
    draws = torch.rand((B, 3), dtype=torch.float64, generator=torch.Generator().manual_seed(5)).numpy()
    ev = lambda: torch.cuda.Event(enable_timing=True)

    def launch(pos, flow, d):
        e0, e1 = ev(), ev()
        e0.record()
        out, _ = fe.mask_pose(pos, flow, off, h_off, draws=d)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1), out[:, 25].cpu().numpy(), out.cpu().numpy()

    def permuted(k, perm):
        p = torch.as_tensor(perm, device=dev)
        pos, flow = data[k]
        return (pos.view(B, N, 3)[p].reshape(B * N, 3).contiguous(),
                flow.view(B, N, 3)[p].reshape(B * N, 3).contiguous())

    launch(*data[0], draws)                       # warm-up
    rows, prev = [], None
    for k in range(K):
        t_seq, cost, o_seq = launch(*data[k], draws)
        r = dict(k=k, seq_ms=t_seq, cost_mean=float(cost.mean()), cost_max=float(cost.max()))
        own = np.argsort(-cost, kind="stable")
        t_own, _, o_own = launch(*permuted(k, own), draws[own])
        r["own_ms"] = t_own
        r["own_same"] = bool(np.array_equal(o_own, o_seq[own]))
        if prev is not None:
            pp = np.argsort(-prev, kind="stable")
            t_prev, _, o_prev = launch(*permuted(k, pp), draws[pp])
            r["prev_ms"] = t_prev
            r["prev_same"] = bool(np.array_equal(o_prev, o_seq[pp]))
            r["corr_prev"] = float(np.corrcoef(prev, cost)[0, 1])
        prev = cost
        rows.append(r)
        print(json.dumps({a: (round(b, 3) if isinstance(b, float) else b) for a, b in r.items()}), flush=True)
    # 3 streams, K - 1 steps, sequence order vs previous-step order (the copies made up front)
    S = 3
    fes = [ssf.Frontend(64, device=0) for _ in range(S)]
    for f in fes:
        f.reserve(B, N)
    st = [torch.cuda.Stream(dev) for _ in range(S)]
    costs = [None] * K
    for k in range(K):
        _, costs[k], _ = launch(*data[k], draws)
    perms = [np.argsort(-costs[k - 1], kind="stable") for k in range(1, K)]
    ordered = [(*permuted(k, pp), draws[pp]) for k, pp in zip(range(1, K), perms)]
    plain = [(*data[k], draws) for k in range(1, K)]
    res = {}
    for name, src in (("seq", plain), ("prev", ordered), ("seq2", plain), ("prev2", ordered)):
        for j in range(S):                        # warm-up every context
            with torch.cuda.stream(st[j]):
                fes[j].mask_pose(src[0][0], src[0][1], off, h_off, draws=src[0][2])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for j, (pos, flow, d) in enumerate(src):
            with torch.cuda.stream(st[j % S]):
                fes[j % S].mask_pose(pos, flow, off, h_off, draws=d)
        torch.cuda.synchronize()
        res[name] = len(src) * B / (time.perf_counter() - t0)
        print(name, round(res[name]), flush=True)
    json.dump(dict(rows=rows, overlapped_frames_per_s=res, B=B), open(outp, "w"), indent=1)


if __name__ == "__main__":
    main()
