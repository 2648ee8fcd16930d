"""End-to-end node chain: an npz DATASET_PATH directory replayed through
PointCloudOdometry -> frameFeature -> lidarOdometry_onlyPC with the reference's topic layouts,
/frame_odom1 and /frame_odom2 against the oracle, and the TUM file written from /frame_odom2.

Bars: /frame_odom1 [t, q] and /frame_odom2 accumulated poses within 1e-5 m / 1e-6 rad of the
oracle run with the same seeded RandomState draws and the same warm-start chain."""
import numpy as np
import pytest
import torch

from helpers import frame

pytestmark = pytest.mark.gpu


def _angle(q1, q2):
    d = abs(float(np.dot(q1 / np.linalg.norm(q1), q2 / np.linalg.norm(q2))))
    return 2.0 * np.arccos(min(1.0, d))


def test_run_sequence_matches_oracle(oracle, dev, tmp_path):
    from ssf import io as sio
    from ssf import nodes
    frames = [frame(4, k, n_az=1875) for k in range(4)]
    data = tmp_path / "data"          # the reference loads every file of DATASET_PATH
    data.mkdir()
    for k, f in enumerate(frames):
        np.savez(str(data / f"{k:06d}.npz"), pos1=f[0], gt=f[1])
    tum = str(tmp_path / "traj.txt")
    with torch.cuda.device(dev):
        res = nodes.run_sequence(str(data), tum, seed=123)
    assert res["odom1"].shape == (4, 7) and res["odom2"].shape == (3, 7)

    rs = oracle.LegacyRandomState(123)
    for k, f in enumerate(frames):
        ref = oracle.mask_and_pose(f[0], f[1], rs.random_sample(3))
        assert ref["rc"] == 0
        assert np.abs(res["odom1"][k, 0:3] - ref["t"]).max() < 1e-5
        assert _angle(res["odom1"][k, 3:7], ref["q_xyzw"]) < 1e-6

    planes = [oracle.extract_planes(f[0], 64) for f in frames]
    q_rel, t_rel = np.array([0.0, 0, 0, 1]), np.zeros(3)
    q_abs, t_abs = np.array([0.0, 0, 0, 1]), np.zeros(3)
    for k in range(1, len(frames)):
        q_rel, t_rel, _, _ = oracle.register_pair(planes[k - 1], planes[k], 0.05, mode=oracle.MODE_CERES_LM,
                                                  max_iter=8, q_init=q_rel, t_init=t_rel)
        q_abs, t_abs = oracle.accumulate(q_abs, t_abs, q_rel, t_rel)
        got = res["odom2"][k - 1]
        assert np.abs(got[0:3] - t_abs).max() < 1e-5, k
        assert _angle(got[3:7], q_abs) < 1e-6, k

    stamps, t, q = sio.read_tum(tum)
    assert stamps == ["0.100000000", "0.200000000", "0.300000000"]
    assert np.abs(t - res["odom2"][:, 0:3]).max() <= 5e-7 and np.abs(q - res["odom2"][:, 3:7]).max() <= 5e-7


def test_nodes_message_layouts(dev):
    """/plane_frame_cloud1 and /plane_frame_cloud2 carry the PointXYZI layout with the input's
    stamp in frame "map"; /org_frame_cloud1 republishes the input; /frame_odom2 is an
    Odometry in "map" / "map_child"; the plane cloud equals Frontend.extract_planes."""
    from ssf import io as sio
    from ssf import nodes
    bus = nodes.Bus(keep=4)
    ff = nodes.FrameFeatureNode(bus.publish, device=dev)
    lo = nodes.LidarOdometryNode(bus.publish, device=dev)
    bus.subscribe("/velodyne_points", ff.on_cloud)
    bus.subscribe("/plane_frame_cloud1", lo.on_plane_cloud)
    clouds = [frame(2, k, n_az=1875)[0] for k in range(2)]
    for k, c in enumerate(clouds):
        bus.publish("/velodyne_points", sio.xyz_to_cloud(c, stamp=(5, k), frame_id="livox_frame"))
    pc1 = bus.log["/plane_frame_cloud1"]
    assert len(pc1) == 2 and pc1[1].point_step == 32 and pc1[1].header.frame_id == "map"
    assert sio.stamp_of(pc1[1].header) == (5, 1)
    ref = ff.fe.extract_planes(torch.from_numpy(clouds[1]).to(dev)).cpu().numpy()
    assert np.array_equal(sio.cloud_xyzi(pc1[1]), ref)
    org = bus.log["/org_frame_cloud1"][1]
    assert org.header.frame_id == "map" and org.data == sio.xyz_to_cloud(clouds[1]).data
    assert len(bus.log["/frame_odom2"]) == 1          # the first frame only becomes the last frame
    od = bus.log["/frame_odom2"][0]
    assert od.header.frame_id == "map" and od.child_frame_id == "map_child"
    assert len(bus.log["/frame_odom_path2"][-1].poses) == 1
    assert np.array_equal(sio.cloud_xyzi(bus.log["/plane_frame_cloud2"][0]), ref)


def test_map_optimization_node_chain(dev, tmp_path):
    """mapOptmization on the bus (/plane_frame_cloud2 + /frame_odom2 -> /map_odom_res3 and the
    RESULT_PATH TUM file, src/mapOptmization.cpp:355-374, 429-467): with no loop in a short
    forward sequence, trans_loop_adjust stays identity and the map pose is /frame_odom2."""
    from ssf import io as sio
    from ssf import nodes
    frames = [frame(5, k, n_az=900) for k in range(4)]
    data = tmp_path / "data"
    data.mkdir()
    for k, f in enumerate(frames):
        np.savez(str(data / f"{k:06d}.npz"), pos1=f[0], gt=f[1])
    tum2, tum3 = str(tmp_path / "odom2.txt"), str(tmp_path / "map.txt")
    with torch.cuda.device(dev):
        res = nodes.run_sequence(str(data), tum2, seed=7, map_tum_path=tum3)
    assert res["loops"] == []
    s2, t2, q2 = sio.read_tum(tum2)
    s3, t3, q3 = sio.read_tum(tum3)
    assert s2 == s3 and len(s3) == 3
    assert np.abs(t3 - t2).max() <= 1e-6
    for a, b in zip(q2, q3):
        assert _angle(a, b) < 1e-6
