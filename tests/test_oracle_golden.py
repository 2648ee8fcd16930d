"""Pin the CPU oracle to the reference: golden vectors produced by importing the reference's
own scripts/PointCloudOdometry_noSeg.py (+ the sklearn it calls), see tests/golden/make_golden.py."""
import glob
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_mt19937_stream(oracle):
    g = np.load(os.path.join(GOLDEN, "mt19937_ref.npz"))
    for k in g.files:
        rs = oracle.LegacyRandomState(int(k[4:]))
        assert np.array_equal(rs.random_sample(8), g[k])


def test_slove_RT_by_SVD(oracle):
    g = np.load(os.path.join(GOLDEN, "kabsch_ref.npz"))
    for c in range(4):
        rc, R, t = oracle.kabsch(g[f"src{c}"], g[f"dst{c}"])
        assert rc == 0
        assert np.abs(R - g[f"R{c}"]).max() < 1e-12
        assert np.abs(t - g[f"t{c}"]).max() < 1e-12
    rc, _, _ = oracle.kabsch(g["refl_src"], g["refl_dst"])
    assert rc == -2 and int(g["refl_raises_typeerror"]) == 1


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "gmm_noseg_case*.npz"))))
def test_gmm_mask_and_pose(oracle, path):
    g = np.load(path)
    res = oracle.mask_and_pose(g["pos1"], g["flow"], g["draws"])
    info = res["info"]
    assert [int(info["center0"]), int(info["center1"])] == [int(v) for v in g["kmeans_pp_idx"]]
    assert int(info["kmeans_iter"]) == int(g["kmeans_n_iter"])
    assert int(info["em_iter"]) == int(g["gmm_n_iter"])
    assert np.array_equal(res["labels"], g["labels"])
    assert int(info["bg_label"]) == int(g["bg_label"])
    assert np.abs(res["means"] - g["gmm_means"]).max() < 1e-8
    assert abs(info["lower_bound"] - float(g["gmm_lower_bound"])) < 1e-9
    assert np.abs(res["R"] - g["R"]).max() < 1e-12
    assert np.abs(np.r_[res["t"], res["q_xyzw"]] - g["para_t_q"]).max() < 1e-12
