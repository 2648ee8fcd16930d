"""Reference-named entry points (SURVEY §8(b) process surface): the `type=` targets of
launch/*.launch exist as executables, refuse cleanly without rospy (absent in this image) unless
given a dataset to replay offline, and the rospy message conversions keep the reference's
layouts.  CPU only: stand-in message modules replace sensor_msgs / std_msgs / nav_msgs /
geometry_msgs, whose real versions are not installed."""
import os
import subprocess
import sys
import types

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS = os.path.join(REPO, "ssf-slam_amd", "scripts")
# every node type the reference's launch files start (launch/run_*.launch)
LAUNCH_TYPES = ["PointCloudOdometry_noSeg.py", "PointCloudOdometry.py", "PointCloudOdometry_onlyPC.py",
                "frameFeature", "lidarOdometry", "lidarOdometry_onlyPC", "mapOptmization"]


@pytest.mark.parametrize("exe", LAUNCH_TYPES)
def test_launch_targets_exist_and_refuse_without_ros(exe):
    path = os.path.join(SCRIPTS, exe)
    assert os.access(path, os.X_OK)
    # roslaunch appends __name:= / __log:= arguments: they must not break the parser
    r = subprocess.run([sys.executable, path, "__name:=x", "__log:=/tmp/x.log"], capture_output=True,
                       text=True, timeout=120, env=dict(os.environ, HIP_VISIBLE_DEVICES=""))
    assert r.returncode != 0
    assert "rospy is not importable" in r.stderr


def _fake_ros():
    class Obj:
        def __init__(self, *a, **k):
            for key, v in k.items():
                setattr(self, key, v)

    class Time:
        def __init__(self, secs=0, nsecs=0):
            self.secs, self.nsecs = secs, nsecs

    class PointField:
        def __init__(self, name, offset, datatype, count):
            self.name, self.offset, self.datatype, self.count = name, offset, datatype, count

    class Vec:
        def __init__(self):
            self.x = self.y = self.z = 0.0

    class Quat(Vec):
        def __init__(self):
            super().__init__()
            self.w = 1.0

    class Pose:
        def __init__(self):
            self.position, self.orientation = Vec(), Quat()

    class Odometry:
        def __init__(self):
            self.header, self.child_frame_id = None, ""
            self.pose = Obj(pose=Pose())

    class Path:
        def __init__(self):
            self.header, self.poses = None, []

    rospy = types.SimpleNamespace(Time=Time)
    sensor = types.SimpleNamespace(PointCloud2=Obj, PointField=PointField)
    std = types.SimpleNamespace(Header=Obj, Float64MultiArray=Obj)
    nav = types.SimpleNamespace(Odometry=Odometry, Path=Path)
    geo = types.SimpleNamespace(Pose=Pose, PoseStamped=Obj)
    return rospy, sensor, std, nav, geo


def test_ros_message_conversions():
    from ssf import io as sio
    from ssf import nodes, rosbridge
    rospy, sensor, std, nav, geo = _fake_ros()
    xyzi = np.arange(40, dtype=np.float32).reshape(10, 4)
    cloud = sio.xyzi_to_cloud(xyzi, stamp=(7, 123), frame_id="map")
    m = rosbridge.to_ros_cloud(rospy, std, sensor, cloud)
    assert m.point_step == 32 and m.width == 10 and m.header.frame_id == "map"
    assert (m.header.stamp.secs, m.header.stamp.nsecs) == (7, 123)
    assert [(f.name, f.offset) for f in m.fields] == [("x", 0), ("y", 4), ("z", 8), ("intensity", 16)]
    assert np.array_equal(sio.cloud_xyzi(m), xyzi)       # the node classes read the ROS message as is
    od = nodes.Odometry(sio.Header(3, 4, "map"), "map_child",
                        nodes.Pose((1.0, 2.0, 3.0), (0.0, 0.0, 0.6, 0.8)))
    ro = rosbridge.to_ros_odometry(rospy, std, nav, geo, od)
    assert ro.child_frame_id == "map_child" and ro.pose.pose.orientation.z == 0.6
    back = rosbridge.from_ros_odometry(ro)
    assert back.pose.position == (1.0, 2.0, 3.0) and back.pose.orientation == (0.0, 0.0, 0.6, 0.8)
    assert sio.stamp_of(back.header) == (3, 4)
    path = nodes.Path(sio.Header(3, 4, "map"), [(sio.Header(3, 4, "map"), od.pose)] * 2)
    rp = rosbridge.to_ros_path(rospy, std, nav, geo, path)
    assert len(rp.poses) == 2 and rp.poses[1].pose.position.y == 2.0
    arr = rosbridge.to_ros_array(std, nodes.Float64MultiArray([1, 2, 3, 0, 0, 0, 1]))
    assert arr.data == [1.0, 2.0, 3.0, 0.0, 0.0, 0.0, 1.0]


def test_rosbridge_not_available_here():
    from ssf import rosbridge
    assert not rosbridge.available()
    with pytest.raises(SystemExit):
        rosbridge.require()
