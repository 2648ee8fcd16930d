"""CPU-baseline legs for bench.py (TEST INFRASTRUCTURE: the CPU oracle is timed here as the
reported baseline; nothing in the product path imports this module).

Leg "oracle": one synthetic sequence through the C restatement of the reference front-end --
GMM mask + Kabsch (PointCloudOdometry_noSeg.py:97-125), frameFeature (frameFeature.cpp:45-123),
plane table + registration of the pair (lidarOdometry_onlyPC.cpp:147-252) with the warm start
chained -- single-threaded, for a bounded number of seconds.  bench.py starts one process per
core for the all-cores figure (the reference nodes are single-threaded).

Leg "sklearn": the reference's own mask call on this host, GaussianMixture(n_components=2)
.fit_predict on [flow, xyz] (sklearn, third-party; PointCloudOdometry_noSeg.py:97-103), plus the
numpy Kabsch of slove_RT_by_SVD (:19-37, restated: the reference script itself cannot travel).

Usage: python -m oracle.cpu_leg {oracle|sklearn} --seq S --seconds T [--rows R --n-az A ...]
prints one JSON line {"frames": n, "seconds": s, ...}.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "ssf-slam_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def _frames(seq, rows, n_az, n, layout="azimuth"):
    import torch
    torch.set_num_threads(1)
    from ssf import synth
    sc = synth.Scene(seq)
    out = []
    for k in range(n):
        f = synth.scan(seq, k, n_rows=rows, n_az=n_az, scene=sc, layout=layout)
        out.append((f["pos1"].numpy(), f["flow"].numpy()))
    return out


def leg_oracle(a):
    import numpy as np
    from oracle import oracle as O
    O.lib()
    fr = _frames(a.seq, a.rows, a.n_az, 4, a.layout)
    prof = O.profile(a.rows)
    mode = O.MODE_GN if a.solver == "gn" else O.MODE_CERES_LM
    last = O.extract_planes(fr[0][0], a.rows)
    q, t = np.array([0, 0, 0, 1.0]), np.zeros(3)
    done = 0
    t0 = time.perf_counter()
    while True:
        p, f = fr[1 + done % 3]
        O.mask_and_pose(p, f, [0.3, 0.6, 0.9])
        curr = O.extract_planes(p, a.rows)
        q, t, _, _ = O.register_pair(last, curr, prof.plane_max, mode=mode, max_iter=a.iters,
                                     q_init=q, t_init=t)
        last = curr
        done += 1
        el = time.perf_counter() - t0
        if (el >= a.seconds and done >= 1) or el > 4 * a.seconds + 30:
            break
    return dict(frames=done, seconds=el)


def kabsch_np(src, dst):
    """slove_RT_by_SVD (PointCloudOdometry_noSeg.py:19-37), numpy, det > 0 branch."""
    import numpy as np
    ms, md = src.mean(0), dst.mean(0)
    H = (src - ms).T @ (dst - md)
    U, S, Vt = np.linalg.svd(H)
    R = Vt.T @ U.T
    return R, -R @ ms + md


def leg_sklearn(a):
    import numpy as np
    try:
        from sklearn.mixture import GaussianMixture
        import sklearn
    except ImportError as e:                       # not installed on this host
        return dict(frames=0, seconds=0.0, skipped=str(e))
    fr = _frames(a.seq, a.rows, a.n_az, 2, a.layout)
    done = 0
    t0 = time.perf_counter()
    while True:
        p, f = fr[done % 2]
        p = p.astype(np.float64)
        f = f.astype(np.float64)
        np.random.seed(1234 + done)
        lab = GaussianMixture(n_components=2).fit_predict(np.concatenate((f, p), axis=1))
        vals, cnt = np.unique(lab, return_counts=True)
        bg = lab == vals[np.argmax(cnt)]
        kabsch_np(p[bg] + f[bg], p[bg])
        done += 1
        el = time.perf_counter() - t0
        if el >= a.seconds or el > 60:
            break
    return dict(frames=done, seconds=el, sklearn=sklearn.__version__)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("leg", choices=["oracle", "sklearn"])
    ap.add_argument("--seq", type=int, default=0)
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--rows", type=int, default=64)
    ap.add_argument("--n-az", type=int, default=1875)
    ap.add_argument("--layout", default="azimuth", choices=["azimuth", "carla"])
    ap.add_argument("--solver", default="gn")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cpu", type=int, default=None, help="pin this process to one CPU")
    a = ap.parse_args()
    if a.cpu is not None and hasattr(os, "sched_setaffinity"):
        os.sched_setaffinity(0, {a.cpu})
    r = leg_oracle(a) if a.leg == "oracle" else leg_sklearn(a)
    r["leg"] = a.leg
    r["seq"] = a.seq
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
