"""CPU oracle of the TFlow point-set operators (oracle/pn2_oracle.c) against golden vectors
produced by the reference's own torch operators (tests/golden/make_golden_pn2.py: imports
scripts/ActiveSceneFlow/utils/utils.py), plus known-answer cases."""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "pn2_ref.npz")


@pytest.fixture(scope="module")
def g():
    return dict(np.load(GOLD))


def test_fps_matches_reference(g):
    got = O.pn2_fps(g["xyz"], g["fps_idx"].shape[1], start=g["fps_start"])
    assert np.array_equal(got, g["fps_idx"])


def test_knn_matches_reference(g):
    new_xyz = np.take_along_axis(g["xyz"], g["fps_idx"][..., None].astype(np.int64), axis=1)
    d, i = O.pn2_knn(int(g["knn_k"]), new_xyz, g["xyz"])
    assert np.array_equal(i, g["knn_idx"])
    # torch's CPU sqrt (vectorised) is not correctly rounded: 0.5 % of its outputs are 1 ulp
    # off the IEEE sqrt of the same squared distance; the indices above are exact.
    np.testing.assert_allclose(d, g["knn_dist"], rtol=2.5e-7, atol=0)


def test_three_nn_matches_reference(g):
    new_xyz = np.take_along_axis(g["xyz"], g["fps_idx"][..., None].astype(np.int64), axis=1)
    d, i = O.pn2_knn(3, g["xyz"], new_xyz)
    assert np.array_equal(i, g["three_idx"])
    np.testing.assert_allclose(d, g["three_dist"], rtol=2.5e-7, atol=0)


def test_gather_and_group_match_reference(g):
    assert np.array_equal(O.pn2_gather(g["feat"], g["fps_idx"]), g["gathered"])
    assert np.array_equal(O.pn2_gather(g["feat"], g["knn_idx"]), g["grouped"])


def test_three_interpolate_matches_reference(g):
    got = O.pn2_three_interpolate(g["sfeat"], g["three_idx"], g["three_weight"])
    np.testing.assert_allclose(got, g["interp"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("k", [3, 5])
def test_upsample_flow_matches_reference(g, k):
    xyz = np.ascontiguousarray(g["xyz"].transpose(0, 2, 1))
    new_xyz = np.take_along_axis(g["xyz"], g["fps_idx"][..., None].astype(np.int64), axis=1)
    sxyz = np.ascontiguousarray(new_xyz.transpose(0, 2, 1))
    got = O.pn2_upsample_flow(xyz, sxyz, g["sflow"], k=k)
    np.testing.assert_allclose(got, g[f"up{k}"], rtol=1e-5, atol=1e-6)


def test_known_answers():
    # a line of points: FPS from 0 picks the far end, then the middle
    x = np.zeros((1, 5, 3), np.float32)
    x[0, :, 0] = [0, 1, 2, 3, 4]
    assert O.pn2_fps(x, 3).tolist() == [[0, 4, 2]]
    # equal distances: the lower index first (torch.max / stable top-k)
    d, i = O.pn2_knn(2, np.zeros((1, 1, 3), np.float32),
                     np.array([[[1, 0, 0], [-1, 0, 0], [0, 0.5, 0]]], np.float32))
    assert i.tolist() == [[[2, 0]]] and np.allclose(d, [[[0.5, 1.0]]])
    # coincident dense / sparse point: distance clamped at 1e-10 dominates the weights
    xyz = np.zeros((1, 3, 1), np.float32)
    sx = np.array([[[0.0, 1.0, 2.0], [0, 0, 0], [0, 0, 0]]], np.float32)
    sf = np.array([[[7.0, 1.0, 1.0]]], np.float32)
    assert np.allclose(O.pn2_upsample_flow(xyz, sx, sf, k=3), 7.0)
