"""Loop-closure host logic and oracle known answers (CPU only, no GPU).

pcl::getTransformation / getTranslationAndEulerAngles round trips, the quaternion pose of
/frame_odom2, the VoxelGrid and ICP oracle restatements on inputs with known answers, and the
keyframe / loop-detection rules of mapOptmization.cpp:129-197."""
import math

import numpy as np


def test_euler_round_trip():
    from ssf import loop
    rng = np.random.default_rng(0)
    for _ in range(50):
        x, y, z = rng.uniform(-50, 50, 3)
        r, p, yw = rng.uniform(-1.2, 1.2, 3)
        T = loop.get_transformation(x, y, z, r, p, yw)
        assert np.allclose(T[:3, :3] @ T[:3, :3].T, np.eye(3), atol=1e-12)
        got = loop.get_translation_and_euler_angles(T)
        assert np.allclose(got, (x, y, z, r, p, yw), atol=1e-12)


def test_pose_from_quat_matches_euler():
    from ssf import loop
    yaw = 0.3
    q = (0.0, 0.0, math.sin(yaw / 2), math.cos(yaw / 2))
    T = loop.pose_from_quat(q, (1, 2, 3))
    assert np.allclose(T, loop.get_transformation(1, 2, 3, 0, 0, yaw), atol=1e-12)


def test_oracle_voxel_grid_known_centroids(oracle):
    pts = np.array([[0.01, 0.01, 0.01, 1], [0.03, 0.05, 0.02, 3],      # same 0.1 voxel
                    [0.15, 0.01, 0.01, 5],                              # next in x
                    [0.01, 0.15, 0.01, 7]], np.float32)                 # next in y
    out = oracle.voxel_grid(pts, 0.1)
    assert out.shape == (3, 4)
    assert np.allclose(out[0], [0.02, 0.03, 0.015, 2], atol=1e-7)
    assert np.allclose(out[1], pts[2]) and np.allclose(out[2], pts[3])   # voxel index order


def test_oracle_icp_recovers_rigid_motion(oracle):
    rng = np.random.default_rng(1)
    src = np.concatenate([rng.uniform(-10, 10, (1500, 3)), np.zeros((1500, 1))], 1).astype(np.float32)
    a = 0.04
    R = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
    tgt = src.copy()
    tgt[:, :3] = (src[:, :3].astype(np.float64) @ R.T + [0.2, 0.1, -0.3]).astype(np.float32)
    r = oracle.icp(src, tgt)
    assert r["converged"] and r["fitness"] < 1e-8
    assert np.abs(r["T"][:3, :3] - R).max() < 1e-5 and np.abs(r["T"][:3, 3] - [0.2, 0.1, -0.3]).max() < 1e-4


def test_oracle_icp_iteration_cap_and_no_correspondences(oracle):
    rng = np.random.default_rng(2)
    src = np.concatenate([rng.uniform(-5, 5, (400, 3)), np.zeros((400, 1))], 1).astype(np.float32)
    tgt = src + np.array([3, 0, 0, 0], np.float32)
    r = oracle.icp(src, tgt, max_iter=2)
    assert r["state"] == "iterations" and r["iterations"] == 2 and r["converged"]
    r = oracle.icp(src, tgt + 1000, max_corr_dist=1.0)
    assert r["state"] == "no_correspondences" and not r["converged"]


class _NoGpu:
    device = None


def test_keyframe_and_loop_detection_rules():
    from ssf import loop
    lc = loop.LoopCloser(_NoGpu())
    assert lc.is_key_frame(np.eye(4))
    lc.key6d.append([0, 0, 0, 0, 0, 0, 0.0])
    assert not lc.is_key_frame(loop.get_transformation(0.5, 0, 0, 0, 0, 0.005))   # small motion
    assert lc.is_key_frame(loop.get_transformation(1.5, 0, 0, 0, 0, 0))
    assert lc.is_key_frame(loop.get_transformation(0, 0, 0, 0, 0, 0.02))
    # loop detection: nearest keyframe within 15 m whose time differs by > 20 s
    for k, (x, t) in enumerate([(5, 1.0), (10, 2.0), (20, 3.0), (40, 4.0), (6, 30.0)]):
        lc.key6d.append([x, 0, 0, 0, 0, 0, t])
    ids = lc.detect_loop()
    assert ids == (5, 1)            # key 1 (x=5) is nearest to x=6 among the old ones
    assert lc.loop_record_index == 7
    lc.loop_index[5] = 1
    assert lc.detect_loop() is None  # already closed
