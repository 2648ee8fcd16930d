"""Golden vectors for the ASF block in float32: the reference's
scripts/ActiveSceneFlow/main_sju_occ_ros.py:256-284 runs the noSeg mask + Kabsch block on the
network's float32 output -- `points` / `move_gt` are float32 numpy arrays (:226-230), so sklearn
fits the GaussianMixture in float32, `points + move_gt` is a float32 add and slove_RT_by_SVD
(imported from the reference's PointCloudOdometry_noSeg.py, the text-identical function) runs on
float32 arrays.

Run in the build container only (reads /root/reference); the .npz it writes is what the tests read.
pyquaternion is absent: `Quaternion(matrix=R)` (:278) is not called.  Its orthogonality test
(np.allclose(R R^T, I, rtol=1e-05, atol=1e-08), pyquaternion 0.9.9 `_from_matrix`) is restated
on the float32 R and stored as `quat_would_raise` (parity unpinned for that step).

Inputs: 8192-point subsamples (the ASF input size) of seeded synthetic frames (ssf.synth).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import frame_inputs, import_reference  # noqa: E402


def main():
    from collections import Counter
    from sklearn.mixture import GaussianMixture
    ref = import_reference()
    rng = np.random.default_rng(31)
    out = {}
    for case, (seq, frame, seed) in enumerate([(3, 1, 101), (4, 2, 202), (5, 4, 303), (6, 6, 404)]):
        pos1, flow, _ = frame_inputs(seq, frame, 8192, rng)
        points, move_gt = pos1.astype(np.float32), flow.astype(np.float32)   # :226-230
        X = np.concatenate((move_gt, points), axis=1)                        # :257
        assert X.dtype == np.float32
        np.random.seed(seed)
        draws = np.random.random_sample(3)
        np.random.seed(seed)
        model = GaussianMixture(n_components=2)                              # :258
        labels = model.fit_predict(X)                                        # :261
        bg_label = Counter(labels).most_common(1)[0][0]                      # :262
        bg_index = np.argwhere(labels == bg_label).flatten()                 # :263
        target = points[bg_index] + move_gt[bg_index]                        # :274 (f32 add)
        source = points[bg_index]                                            # :275
        R, t = ref.slove_RT_by_SVD(target, source)                           # :277
        would_raise = not np.allclose(np.dot(R, R.conj().transpose()), np.eye(3), rtol=1e-05, atol=1e-08)
        out.update({f"pos1_{case}": points, f"flow_{case}": move_gt, f"draws_{case}": draws,
                    f"labels_{case}": labels.astype(np.uint8), f"bg_label_{case}": np.array(bg_label),
                    f"means_dtype_f32_{case}": np.array(model.means_.dtype == np.float32),
                    f"n_iter_{case}": np.array(model.n_iter_), f"R_{case}": R, f"t_{case}": t.ravel(),
                    f"quat_would_raise_{case}": np.array(would_raise)})
        print(f"case{case}: X {X.dtype} means {model.means_.dtype} R {R.dtype} iter {model.n_iter_} "
              f"bg {len(bg_index)} quat_would_raise {would_raise}")
    np.savez_compressed(os.path.join(HERE, "gmm_asf_f32.npz"), **out)


if __name__ == "__main__":
    main()
