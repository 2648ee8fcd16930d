"""Main functions of the reference-named executables in `ssf-slam_amd/scripts/` -- the `type=`
targets of launch/*.launch (SURVEY §8(b) process surface):

  PointCloudOdometry_noSeg.py / PointCloudOdometry.py / PointCloudOdometry_onlyPC.py
      node velodyne_points_odometry_node, param ~DATASET_PATH, 10 Hz replay of the npz frames
      (scripts/PointCloudOdometry_noSeg.py:38-127, PointCloudOdometry.py:36-105,
      PointCloudOdometry_onlyPC.py:14-65)
  frameFeature, lidarOdometry_onlyPC, lidarOdometry, mapOptmization
      the C++ nodes (src/frameFeature.cpp:141-168, lidarOdometry_onlyPC.cpp:313-334,
      lidarOdometry.cpp:207-230, mapOptmization.cpp:457-485) as Python hosts over the C ABI.

With rospy importable they run as ROS1 nodes with the reference's names, topics and params.
rospy is absent from this image: then the PointCloudOdometry scripts take `--dataset PATH` and
replay the whole launch graph in-process (ssf.nodes.run_sequence), and the C++-node executables
say how to do that.  roslaunch appends `__name:=...` / `__log:=...` arguments, so every parser
uses parse_known_args, as the reference's ASF scripts do (main_sju_occ_ros.py:495-566).
"""
from __future__ import annotations

import argparse
import json

SOURCE_MODES = {  # script -> (data-source mode, launch graph of the offline replay)
    "PointCloudOdometry_noSeg.py": ("gmm", "noSeg"),
    "PointCloudOdometry.py": ("gt", "Seg"),
    "PointCloudOdometry_onlyPC.py": ("none", "onlyPC"),
}


def _parser(prog):
    ap = argparse.ArgumentParser(prog=prog)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--rows", type=int, default=64, choices=[16, 64], help="N_SCAN_ROW profile")
    return ap


def pointcloud_odometry_main(script: str, argv=None):
    mode, launch = SOURCE_MODES[script]
    ap = _parser(script)
    ap.add_argument("--dataset", default=None,
                    help="offline: replay this DATASET_PATH through the whole run_%s.launch graph" % launch)
    ap.add_argument("--result", default=None, help="offline: RESULT_PATH TUM file (appended)")
    ap.add_argument("--seed", type=int, default=None, help="np.random.seed for the GMM k-means++")
    ap.add_argument("--rate", type=float, default=10.0, help="publish rate (rospy.Rate(10), :44)")
    a, _ = ap.parse_known_args(argv)
    from . import rosbridge
    if a.dataset is None and rosbridge.available():
        return _ros_pointcloud_odometry(a, mode)
    if a.dataset is None:
        raise SystemExit(f"{script}: rospy is not importable; pass --dataset DATASET_PATH to replay "
                         f"the run_{launch}.launch graph offline")
    import torch
    from .nodes import run_sequence
    torch.cuda.set_device(a.device)
    res = run_sequence(a.dataset, a.result, n_rows=a.rows, seed=a.seed, launch=launch,
                       rate_hz=a.rate)
    print(json.dumps({"script": script, "launch": launch, "frames": len(res["stamps"]),
                      "frame_odom1": res["odom1"].tolist(), "frame_odom2": res["odom2"].tolist()}))
    return res


def _ros_pointcloud_odometry(a, mode):
    import torch
    from . import io as sio
    from . import rosbridge
    from .nodes import PointCloudOdometryNode
    rospy = rosbridge.require()[0]
    rospy.init_node("velodyne_points_odometry_node", anonymous=True)
    topics = ["/velodyne_points"] + ([] if mode == "none" else ["/frame_odom1"])
    # PointCloudOdometry_onlyPC.py:15 advertises velodyne_points with queue 10, the others 100
    pub = rosbridge.RosPublisher(topics, queue={"/velodyne_points": 10} if mode == "none" else None)
    rate = rospy.Rate(a.rate)
    rospy.loginfo("\033[1;32m----> PointCloudOdometry Started.\033[0m")
    root = rospy.get_param("~DATASET_PATH") if rospy.has_param("~DATASET_PATH") else "."
    torch.cuda.set_device(a.device)
    node = PointCloudOdometryNode(pub, device=a.device, mode=mode, seed=a.seed)
    keys = ("pos1",) if mode == "none" else ("pos1", "gt") + (("s_fg_mask",) if mode == "gt" else ())
    for path in sio.sequence_files(root):
        if rospy.is_shutdown():
            break
        rospy.loginfo(path)
        fr = sio.load_frame(path, keys)
        now = rospy.Time.now()
        node.on_frame(fr["pos1"], fr.get("gt"), (now.secs, now.nsecs),
                      gt_mask=fr.get("s_fg_mask") if mode == "gt" else None)
        rate.sleep()


NODES = {  # executable -> (ROS node name, reference main)
    "frameFeature": ("frameFeature", "src/frameFeature.cpp:154-168"),
    "lidarOdometry_onlyPC": ("LidarOdometry", "src/lidarOdometry_onlyPC.cpp:313-334"),
    "lidarOdometry": ("LidarOdometry", "src/lidarOdometry.cpp:207-230"),
    "mapOptmization": ("mapOptmization", "src/mapOptmization.cpp:457-485"),
}


def node_main(exe: str, argv=None):
    """The C++ node executables: subscribe / process / publish until shutdown."""
    ap = _parser(exe)
    ap.add_argument("--solver", default="ceres_lm", choices=["ceres_lm", "gn"])
    a, _ = ap.parse_known_args(argv)
    from . import rosbridge
    if not rosbridge.available():
        raise SystemExit(f"{exe}: rospy is not importable.  Offline, the launch graphs run in one "
                         f"process: `python -m ssf.run DATASET_PATH --launch noSeg|Seg|onlyPC` or "
                         f"scripts/PointCloudOdometry*.py --dataset DATASET_PATH")
    import torch
    from . import nodes
    rospy, sensor_msgs, std_msgs, nav_msgs, _ = rosbridge.require()
    name, _ref = NODES[exe]
    rospy.init_node(name)
    torch.cuda.set_device(a.device)
    if exe == "frameFeature":
        pub = rosbridge.RosPublisher(["/plane_frame_cloud1", "/org_frame_cloud1"])
        node = nodes.FrameFeatureNode(pub, n_rows=a.rows, device=a.device)
        rospy.Subscriber("/velodyne_points", sensor_msgs.PointCloud2, node.on_cloud, queue_size=10)
    elif exe in ("lidarOdometry_onlyPC", "lidarOdometry"):
        pub = rosbridge.RosPublisher(["/plane_frame_cloud2", "/frame_odom2", "/frame_odom_path2"])
        if exe == "lidarOdometry_onlyPC":
            node = nodes.LidarOdometryNode(pub, n_rows=a.rows, device=a.device, solver=a.solver)
        else:
            node = nodes.LidarOdometryIngestNode(pub, device=a.device)
            rospy.Subscriber("/frame_odom1", std_msgs.Float64MultiArray, node.on_odom, queue_size=100)
        rospy.Subscriber("/plane_frame_cloud1", sensor_msgs.PointCloud2, node.on_plane_cloud,
                         queue_size=10)
    else:
        path = rospy.get_param("~RESULT_PATH") if rospy.has_param("~RESULT_PATH") else None
        pub = rosbridge.RosPublisher(["/map_odom_res3", "/map_frame_res3", "/map_laser_path_res3"])
        node = nodes.MapOptimizationNode(pub, device=a.device, tum_path=path)
        rospy.Subscriber("/plane_frame_cloud2", sensor_msgs.PointCloud2, node.on_plane_cloud,
                         queue_size=10)                               # mapOptmization.cpp:473
        rospy.Subscriber("/frame_odom2", nav_msgs.Odometry,
                         lambda m: node.on_odom(rosbridge.from_ros_odometry(m)), queue_size=100)
    rospy.loginfo(f"\033[1;32m----> {name} Started.\033[0m")
    rospy.spin()
