"""End-to-end node chains (SURVEY §8(b) process surface, §8(f) rows 1-2): an npz DATASET_PATH
directory replayed through the node graphs of launch/run_onlyPC.launch, run_noSeg.launch and
run_Seg.launch with the reference's topic layouts; /frame_odom1 and /frame_odom2 against the
oracle, and the TUM file appended from /frame_odom2.

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


def _dataset(tmp_path, frames, with_mask=False):
    data = tmp_path / "data"          # the reference loads every file of DATASET_PATH
    data.mkdir()
    for k, f in enumerate(frames):
        extra = dict(s_fg_mask=f[2]) if with_mask else {}
        np.savez(str(data / f"{k:06d}.npz"), pos1=f[0], gt=f[1], **extra)
    return str(data)


def test_run_onlyPC_launch_matches_oracle(oracle, dev, tmp_path):
    """run_onlyPC.launch: PointCloudOdometry_onlyPC (cloud only, no /frame_odom1) ->
    frameFeature -> lidarOdometry_onlyPC (Ceres-LM registration, warm start chained)."""
    from ssf import io as sio
    from ssf import nodes
    frames = [frame(4, k, n_az=1875) for k in range(4)]
    tum = str(tmp_path / "traj.txt")
    with torch.cuda.device(dev):
        res = nodes.run_sequence(_dataset(tmp_path, frames), tum, launch="onlyPC")
    assert res["odom1"].shape == (0, 7) and res["odom2"].shape == (3, 7)
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


@pytest.mark.parametrize("launch", ["noSeg", "Seg"])
def test_run_ssf_launch_matches_oracle(oracle, dev, tmp_path, launch):
    """run_noSeg.launch / run_Seg.launch: PointCloudOdometry_noSeg (GMM mask, seeded) or
    PointCloudOdometry (s_fg_mask == 0) -> Kabsch -> /frame_odom1 [t, q]; frameFeature;
    lidarOdometry (src/lidarOdometry.cpp:145-159, 176-205): the first plane cloud pops nothing,
    plane cloud k pops the queue front -- the pose published with frame k - 1 -- and accumulates
    it.  /frame_odom1 against the oracle's mask + Kabsch, /frame_odom2 against the oracle's
    accumulation of those poses in queue order, and the appended TUM file."""
    from ssf import io as sio
    from ssf import nodes
    frames = [frame(6, k, n_az=1875) for k in range(5)]
    tum = str(tmp_path / "traj.txt")
    with open(tum, "w") as f:                      # RESULT_PATH is appended to, never wiped
        f.write("0.000000000 0.000000 0.000000 0.000000 0.000000 0.000000 0.000000 1.000000\n")
    with torch.cuda.device(dev):
        res = nodes.run_sequence(_dataset(tmp_path, frames, with_mask=True), tum, seed=123,
                                 launch=launch)
    assert res["odom1"].shape == (5, 7) and res["odom2"].shape == (4, 7)
    rs = oracle.LegacyRandomState(123)
    ref_t, ref_q = [], []
    for k, f in enumerate(frames):
        if launch == "noSeg":
            ref = oracle.mask_and_pose(f[0], f[1], rs.random_sample(3))
            assert ref["rc"] == 0
            t_k, q_k = ref["t"], ref["q_xyzw"]
        else:
            bg = f[2] == 0
            rc, R, t_k = oracle.kabsch(f[0].astype(np.float64) + f[1], f[0].astype(np.float64), mask=bg)
            assert rc == 0
            rc, q_k = oracle.quat_from_R(R)
            assert rc == 0
        assert np.abs(res["odom1"][k, 0:3] - t_k).max() < 1e-5, k
        assert _angle(res["odom1"][k, 3:7], q_k) < 1e-6, k
        ref_t.append(np.asarray(t_k)); ref_q.append(np.asarray(q_k))
    q_abs, t_abs = np.array([0.0, 0, 0, 1]), np.zeros(3)
    for k in range(1, len(frames)):                 # plane cloud k <- odometryQueue.front() = pose k - 1
        q_abs, t_abs = oracle.accumulate(q_abs, t_abs, ref_q[k - 1], ref_t[k - 1])
        got = res["odom2"][k - 1]
        assert np.abs(got[0:3] - t_abs).max() < 2e-5, k
        assert _angle(got[3:7], q_abs) < 2e-6, k
    stamps, t, q = sio.read_tum(tum)
    assert stamps == ["0.000000000", "0.100000000", "0.200000000", "0.300000000", "0.400000000"]
    assert np.abs(t[1:] - res["odom2"][:, 0:3]).max() <= 5e-7


def test_ingest_node_empty_queue_raises(dev):
    """A plane cloud that overtakes its pose: the reference reads front() of an empty queue (UB,
    lidarOdometry.cpp:148); the node raises instead of inventing a pose."""
    from ssf import io as sio
    from ssf import nodes
    bus = nodes.Bus(keep=4)
    lo = nodes.LidarOdometryIngestNode(bus.publish, device=dev)
    xyzi = np.zeros((20, 4), np.float32)
    lo.on_plane_cloud(sio.xyzi_to_cloud(xyzi, (0, 0)))        # first cloud: flagStart only
    with pytest.raises(nodes.SSFError):
        lo.on_plane_cloud(sio.xyzi_to_cloud(xyzi, (0, 1)))
    lo.on_odom(nodes.Float64MultiArray([1.0, 2.0, 3.0, 0.0, 0.0, 0.0, 1.0]))
    od = lo.on_plane_cloud(sio.xyzi_to_cloud(xyzi, (0, 2)))
    assert od.pose.position == (1.0, 2.0, 3.0) and od.pose.orientation == (0.0, 0.0, 0.0, 1.0)
    assert len(bus.log["/plane_frame_cloud2"]) == 1


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
    tum2, tum3 = str(tmp_path / "odom2.txt"), str(tmp_path / "map.txt")
    with torch.cuda.device(dev):
        res = nodes.run_sequence(_dataset(tmp_path, frames), tum2, seed=7, map_tum_path=tum3,
                                 launch="onlyPC")
    assert res["loops"] == []
    s2, t2, q2 = sio.read_tum(tum2)
    s3, t3, q3 = sio.read_tum(tum3)
    assert s2 == s3 and len(s3) == 3
    assert np.abs(t3 - t2).max() <= 1e-6
    for a, b in zip(q2, q3):
        assert _angle(a, b) < 1e-6


def test_entry_script_offline_replay(dev, tmp_path):
    """scripts/PointCloudOdometry_noSeg.py --dataset (no rospy): the run_noSeg.launch graph in one
    process, the same poses as ssf.nodes.run_sequence and the RESULT_PATH TUM file appended."""
    import json
    import os
    import subprocess
    import sys
    from ssf import io as sio
    from ssf import nodes
    frames = [frame(7, k, n_az=900) for k in range(3)]
    data = _dataset(tmp_path, frames)
    tum = str(tmp_path / "r.tum")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = os.path.join(repo, "ssf-slam_amd", "scripts", "PointCloudOdometry_noSeg.py")
    r = subprocess.run([sys.executable, script, "--dataset", data, "--result", tum, "--seed", "5",
                        "__name:=velodyne_points_odometry_node"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["launch"] == "noSeg" and out["frames"] == 3
    with torch.cuda.device(dev):
        res = nodes.run_sequence(data, None, seed=5, launch="noSeg")
    assert np.abs(np.array(out["frame_odom2"]) - res["odom2"]).max() < 1e-12
    assert np.abs(np.array(out["frame_odom1"]) - res["odom1"]).max() < 1e-12
    stamps, t, _ = sio.read_tum(tum)
    assert len(stamps) == 2 and np.abs(t - res["odom2"][:, 0:3]).max() <= 5e-7
