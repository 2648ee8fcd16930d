"""CPU study (numpy, no GPU): how many 64-point blocks a Lloyd skip pass would still have to read
if each block kept a summary of its records.  k-means with k-means++ seeding on
synthetic frames; from pass 4 on, a point is re-read when |g_r| <= B1(t, r)|v| + B2(t, r) (the
kernel's drift bound, without its f32 margins); printed: the fraction of such points and the
fraction of 64-point blocks (frame order) that hold one.
"""
import sys, numpy as np
import os
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'ssf-slam_amd'), REPO]
from ssf import synth
rng = np.random.default_rng(0)
for s in range(6):
    fr = synth.scan(s, 0)
    X = np.concatenate([fr["flow"].numpy(), fr["pos1"].numpy()], 1).astype(np.float64)
    X = X - X.mean(0)
    n = len(X)
    # kmeans++ (2 centres, 2 local trials)
    c0 = X[rng.integers(n)]
    d0 = ((X - c0) ** 2).sum(1)
    cand = np.searchsorted(np.cumsum(d0), rng.random(2) * d0.sum())
    pots = [np.minimum(d0, ((X - X[c]) ** 2).sum(1)).sum() for c in cand]
    c1 = X[cand[int(np.argmin(pots))]]
    C = np.stack([c0, c1])
    vn = np.sqrt((X ** 2).sum(1))
    hist = []
    rec_g = rec_r = None
    lab = None
    out = []
    for it in range(300):
        csn = (C ** 2).sum(1)
        w = C[1] - C[0]; sv = csn[0] - csn[1]
        hist.append((w, sv))
        g = (-2 * X @ C[0] + csn[0]) - (-2 * X @ C[1] + csn[1])   # D0 - D1
        newlab = (g > 0).astype(int)
        if it >= 4:
            B1 = np.array([2 * np.linalg.norm(w - hist[r][0]) for r in range(it + 1)])
            B2 = np.array([abs(sv - hist[r][1]) for r in range(it + 1)])
            fail = np.abs(rec_g) <= B1[rec_r] * vn + B2[rec_r]
            blk = fail[: n // 64 * 64].reshape(-1, 64).any(1)
            out.append((fail.mean(), blk.mean()))
            rec_g = np.where(fail, g, rec_g); rec_r = np.where(fail, it, rec_r)
        else:
            rec_g, rec_r = g.copy(), np.full(n, it)
        changed = lab is None or (newlab != lab).any()
        lab = newlab
        nc = np.stack([X[lab == k].mean(0) for k in range(2)])
        shift = ((nc - C) ** 2).sum()
        C = nc
        if not changed or shift <= 1e-4 * X.var(0).mean():
            break
    if out:
        f = np.array(out)
        print(f"frame {s}: {it+1} Lloyd passes; skip passes {len(out)}: failing points {f[:,0].mean():.3f}, failing 64-blocks {f[:,1].mean():.3f}")
    else:
        print(f"frame {s}: {it+1} passes")
