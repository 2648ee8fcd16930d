"""Generate golden vectors for the Python half of the hot path from the REFERENCE itself.

Run in the build container only (it reads /root/reference, which does not exist on the GPU
box); the resulting .npz files are committed and are what the tests read.

What is imported / called:
  * /root/reference/scripts/PointCloudOdometry_noSeg.py, with the ROS-only modules it imports
    at module level (rospy, sensor_msgs.msg, std_msgs.msg, pyquaternion) replaced by empty
    stubs -- all ROS work sits under `if __name__ == '__main__'` (:40), so importing only
    defines slove_RT_by_SVD (:19-37).
  * sklearn.mixture.GaussianMixture(n_components=2).fit_predict (the call at :98-101), with the
    global numpy RandomState seeded first (the reference leaves random_state=None).
  * sklearn.cluster.KMeans / kmeans_plusplus for the intermediate k-means values.
pyquaternion is not installed (and there is no network), so Quaternion(matrix=R) (:119) is not
imported; q is produced by the restated trace method and marked as such (parity unpinned for
that last step).

Inputs: synthetic frames from ssf.synth (seeded), subsampled to small point counts so the
fixtures stay small.  Each fixture stores inputs + expected outputs only.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SCRIPT = "/root/reference/scripts/PointCloudOdometry_noSeg.py"
sys.path.insert(0, os.path.join(REPO, "ssf-slam_amd"))


def import_reference():
    for name in ("rospy", "sensor_msgs", "sensor_msgs.msg", "std_msgs", "std_msgs.msg",
                 "pyquaternion"):
        mod = types.ModuleType(name)
        sys.modules.setdefault(name, mod)
    sys.modules["sensor_msgs.msg"].PointCloud2 = object
    sys.modules["sensor_msgs.msg"].PointField = object
    sys.modules["std_msgs.msg"].Float64MultiArray = object
    sys.modules["pyquaternion"].Quaternion = None
    spec = importlib.util.spec_from_file_location("ref_noSeg", REF_SCRIPT)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def frame_inputs(seq, frame, n_sub, rng):
    import torch  # noqa: F401
    from ssf import synth
    f = synth.scan(seq, frame)
    pos1 = f["pos1"].numpy()
    flow = f["flow"].numpy()
    fg = f["s_fg_mask"].numpy()
    if n_sub is not None and n_sub < pos1.shape[0]:
        # keep every dynamic point plus a random static subset, original order
        dyn = np.nonzero(fg)[0]
        sta = np.nonzero(fg == 0)[0]
        keep = np.sort(np.concatenate([dyn[: n_sub // 8], rng.choice(sta, n_sub - min(len(dyn), n_sub // 8), replace=False)]))
        pos1, flow, fg = pos1[keep], flow[keep], fg[keep]
    return pos1.astype(np.float32), flow.astype(np.float32), fg.astype(np.uint8)


def quat_trace(R):
    m = R.T
    if m[2, 2] < 0:
        if m[0, 0] > m[1, 1]:
            t = 1 + m[0, 0] - m[1, 1] - m[2, 2]
            q = [m[1, 2] - m[2, 1], t, m[0, 1] + m[1, 0], m[2, 0] + m[0, 2]]
        else:
            t = 1 - m[0, 0] + m[1, 1] - m[2, 2]
            q = [m[2, 0] - m[0, 2], m[0, 1] + m[1, 0], t, m[1, 2] + m[2, 1]]
    else:
        if m[0, 0] < -m[1, 1]:
            t = 1 - m[0, 0] - m[1, 1] + m[2, 2]
            q = [m[0, 1] - m[1, 0], m[2, 0] + m[0, 2], m[1, 2] + m[2, 1], t]
        else:
            t = 1 + m[0, 0] + m[1, 1] + m[2, 2]
            q = [t, m[1, 2] - m[2, 1], m[2, 0] - m[0, 2], m[0, 1] - m[1, 0]]
    q = np.array(q, np.float64) * (0.5 / np.sqrt(t))
    return np.array([q[1], q[2], q[3], q[0]])  # x y z w


def main():
    from sklearn.cluster import KMeans, kmeans_plusplus
    from sklearn.mixture import GaussianMixture
    from collections import Counter

    ref = import_reference()
    rng = np.random.default_rng(7)

    # ---- 1. slove_RT_by_SVD known answers (random rigid transforms + noise)
    ks = {}
    for case, n in enumerate([3, 50, 1000, 4000]):
        g = np.random.default_rng(100 + case)
        src = g.normal(0, 10, (n, 3))
        ang = g.uniform(-0.5, 0.5, 3)
        cx, cy, cz = np.cos(ang); sx, sy, sz = np.sin(ang)
        Rg = (np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]]) @ np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
              @ np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]]))
        tg = g.normal(0, 2, 3)
        dst = src @ Rg.T + tg + g.normal(0, 0.01, (n, 3))
        R, t = ref.slove_RT_by_SVD(src, dst)
        ks[f"src{case}"] = src; ks[f"dst{case}"] = dst; ks[f"R{case}"] = R; ks[f"t{case}"] = t.ravel()
    # reflection case: the reference raises TypeError (`Vt.T & U.T`, :33)
    src = np.random.default_rng(5).normal(0, 1, (20, 3))
    dst = src * np.array([1.0, 1.0, -1.0])
    try:
        ref.slove_RT_by_SVD(src, dst)
        raised = 0
    except TypeError:
        raised = 1
    ks["refl_src"] = src; ks["refl_dst"] = dst; ks["refl_raises_typeerror"] = np.array(raised)
    np.savez_compressed(os.path.join(HERE, "kabsch_ref.npz"), **ks)

    # ---- 2. numpy legacy RandomState stream (what the GMM init consumes)
    mt = {}
    for s in (0, 1234, 20240000, 4294967295):
        np.random.seed(s)
        mt[f"seed{s}"] = np.random.random_sample(8)
    np.savez_compressed(os.path.join(HERE, "mt19937_ref.npz"), **mt)

    # ---- 3. GMM mask + full noSeg block on synthetic frames
    for case, (seq, frame, n_sub, seed) in enumerate([(0, 0, 3000, 11), (1, 3, 6000, 1234),
                                                       (2, 5, 12000, 20240000)]):
        pos1, flow, fg = frame_inputs(seq, frame, n_sub, rng)
        points = pos1.astype(np.float64)        # npz pos1 (f64 on the reference's data path)
        move_gt = flow.astype(np.float64)       # npz gt
        X = np.concatenate((move_gt, points), axis=1)            # :97
        np.random.seed(seed)
        draws = np.random.random_sample(3)
        np.random.seed(seed)
        model = GaussianMixture(n_components=2)                  # :98
        all_label = model.fit_predict(X)                         # :101
        bg_label = Counter(all_label).most_common(1)[0][0]       # :102
        bg_index = np.argwhere(all_label == bg_label).flatten()  # :103
        target = points[bg_index] + move_gt[bg_index]            # :114
        source = points[bg_index]                                # :115
        R, t = ref.slove_RT_by_SVD(target, source)               # :118
        q = quat_trace(R)                                        # :119 (restated, see header)
        para_t_q = np.hstack((t.flatten(), q))                   # :123
        # intermediates
        Xc = X - X.mean(axis=0)
        _, pp_idx = kmeans_plusplus(Xc, 2, random_state=np.random.RandomState(seed))
        km = KMeans(n_clusters=2, n_init=1, random_state=np.random.RandomState(seed)).fit(X)
        np.savez_compressed(
            os.path.join(HERE, f"gmm_noseg_case{case}.npz"),
            pos1=pos1, flow=flow, s_fg_mask=fg, seed=np.array(seed), draws=draws,
            labels=all_label.astype(np.uint8), bg_label=np.array(bg_label),
            gmm_means=model.means_, gmm_n_iter=np.array(model.n_iter_),
            gmm_lower_bound=np.array(model.lower_bound_), gmm_converged=np.array(model.converged_),
            kmeans_pp_idx=pp_idx, kmeans_labels=km.labels_.astype(np.uint8),
            kmeans_centers=km.cluster_centers_, kmeans_n_iter=np.array(km.n_iter_),
            R=R, t=t.ravel(), para_t_q=para_t_q)
        print(f"case{case}: n={len(points)} gmm_iter={model.n_iter_} km_iter={km.n_iter_} "
              f"bg={len(bg_index)} pp={pp_idx}")


if __name__ == "__main__":
    main()
