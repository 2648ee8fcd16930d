"""rospy wiring of the node classes (SURVEY §8(b) process surface): the reference's node names,
topics, queue sizes and parameters, with the in-process stand-in messages of `ssf.io` /
`ssf.nodes` converted to the real ROS message classes on publish.

Import-guarded: rospy, sensor_msgs, std_msgs, nav_msgs and geometry_msgs are NOT in this image,
so `available()` is False here and on the GPU box; every converter takes the message modules as
arguments (defaulting to the real ones), so the conversions are testable with stand-in modules.

Subscribed callbacks need no conversion: the node classes read PointCloud2 / Float64MultiArray
attributes duck-typed (`ssf.io.cloud_points`, `ssf.io.stamp_of`, `msg.data`).
"""
from __future__ import annotations

import importlib


def _mod(name):
    try:
        return importlib.import_module(name)
    except ImportError:
        return None


def available() -> bool:
    return all(_mod(m) is not None for m in ("rospy", "sensor_msgs.msg", "std_msgs.msg",
                                             "nav_msgs.msg", "geometry_msgs.msg"))


def require():
    if not available():
        raise SystemExit("rospy / sensor_msgs / std_msgs / nav_msgs / geometry_msgs are not "
                         "importable: run inside a ROS1 environment, or replay a dataset offline "
                         "with `python -m ssf.run DATASET_PATH --launch noSeg|Seg|onlyPC`")
    return (importlib.import_module("rospy"), importlib.import_module("sensor_msgs.msg"),
            importlib.import_module("std_msgs.msg"), importlib.import_module("nav_msgs.msg"),
            importlib.import_module("geometry_msgs.msg"))


def _stamp(rospy, header):
    from . import io as sio
    sec, nsec = sio.stamp_of(header)
    return rospy.Time(sec, nsec)


def to_ros_header(rospy, std_msgs, header):
    h = std_msgs.Header()
    h.stamp = _stamp(rospy, header)
    h.frame_id = header.frame_id
    return h


def to_ros_cloud(rospy, std_msgs, sensor_msgs, msg):
    """ssf.io.PointCloud2 stand-in -> sensor_msgs/PointCloud2 (same fields, offsets, bytes)."""
    out = sensor_msgs.PointCloud2()
    out.header = to_ros_header(rospy, std_msgs, msg.header)
    out.height, out.width = int(msg.height), int(msg.width)
    out.fields = [sensor_msgs.PointField(f.name, int(f.offset), int(f.datatype), int(f.count))
                  for f in msg.fields]
    out.is_bigendian = bool(msg.is_bigendian)
    out.point_step, out.row_step = int(msg.point_step), int(msg.row_step)
    out.data = bytes(msg.data)
    out.is_dense = bool(msg.is_dense)
    return out


def _ros_pose(geometry_msgs, pose):
    p = geometry_msgs.Pose()
    p.position.x, p.position.y, p.position.z = (float(v) for v in pose.position)
    p.orientation.x, p.orientation.y, p.orientation.z, p.orientation.w = (float(v) for v in pose.orientation)
    return p


def to_ros_odometry(rospy, std_msgs, nav_msgs, geometry_msgs, msg):
    """ssf.nodes.Odometry -> nav_msgs/Odometry (frame "map", child "map_child")."""
    out = nav_msgs.Odometry()
    out.header = to_ros_header(rospy, std_msgs, msg.header)
    out.child_frame_id = msg.child_frame_id
    out.pose.pose = _ros_pose(geometry_msgs, msg.pose)
    return out


def to_ros_path(rospy, std_msgs, nav_msgs, geometry_msgs, msg):
    """ssf.nodes.Path -> nav_msgs/Path of PoseStamped."""
    out = nav_msgs.Path()
    out.header = to_ros_header(rospy, std_msgs, msg.header)
    for hdr, pose in msg.poses:
        ps = geometry_msgs.PoseStamped()
        ps.header = to_ros_header(rospy, std_msgs, hdr)
        ps.pose = _ros_pose(geometry_msgs, pose)
        out.poses.append(ps)
    return out


def from_ros_odometry(msg):
    """nav_msgs/Odometry -> the ssf.nodes.Odometry stand-in the node classes read."""
    from . import io as sio
    from .nodes import Odometry, Pose
    sec, nsec = sio.stamp_of(msg.header)
    p, o = msg.pose.pose.position, msg.pose.pose.orientation
    return Odometry(sio.Header(sec, nsec, msg.header.frame_id), msg.child_frame_id,
                    Pose((p.x, p.y, p.z), (o.x, o.y, o.z, o.w)))


def to_ros_array(std_msgs, msg):
    return std_msgs.Float64MultiArray(data=[float(v) for v in msg.data])


# topic -> (message class attribute path, converter kind); queue sizes from the reference
TOPICS = {
    "/velodyne_points": ("sensor_msgs", "PointCloud2", "cloud", 100),   # PointCloudOdometry_noSeg.py:42
    #                                          (PointCloudOdometry_onlyPC.py:15 uses 10: queue= below)
    "/frame_odom1": ("std_msgs", "Float64MultiArray", "array", 100),    # :42
    "/plane_frame_cloud1": ("sensor_msgs", "PointCloud2", "cloud", 100),  # frameFeature.cpp:162
    "/org_frame_cloud1": ("sensor_msgs", "PointCloud2", "cloud", 100),    # :163
    "/plane_frame_cloud2": ("sensor_msgs", "PointCloud2", "cloud", 100),  # lidarOdometry*.cpp:325
    "/frame_odom2": ("nav_msgs", "Odometry", "odom", 100),                # :326
    "/frame_odom_path2": ("nav_msgs", "Path", "path", 100),               # :327
    "/map_odom_res3": ("nav_msgs", "Odometry", "odom", 100),              # mapOptmization.cpp:471-478
    "/map_frame_res3": ("sensor_msgs", "PointCloud2", "cloud", 10),       # mapOptmization.cpp:475
    "/map_laser_path_res3": ("nav_msgs", "Path", "path", 100),
}


class RosPublisher:
    """publish(topic, stand-in message) -> the real publisher of that topic, converted."""

    def __init__(self, topics, mods=None, queue=None):
        """queue: {topic: size} where the publishing script's own line differs from TOPICS"""
        self.rospy, self.sensor_msgs, self.std_msgs, self.nav_msgs, self.geometry_msgs = mods or require()
        self.pubs = {}
        for t in topics:
            pkg, cls, kind, q = TOPICS[t]
            q = (queue or {}).get(t, q)
            klass = getattr(getattr(self, pkg), cls)
            self.pubs[t] = (self.rospy.Publisher(t.lstrip("/"), klass, queue_size=q), kind)

    def convert(self, kind, msg):
        if kind == "cloud":
            return to_ros_cloud(self.rospy, self.std_msgs, self.sensor_msgs, msg)
        if kind == "array":
            return to_ros_array(self.std_msgs, msg)
        if kind == "odom":
            return to_ros_odometry(self.rospy, self.std_msgs, self.nav_msgs, self.geometry_msgs, msg)
        return to_ros_path(self.rospy, self.std_msgs, self.nav_msgs, self.geometry_msgs, msg)

    def __call__(self, topic, msg):
        ent = self.pubs.get(topic)
        if ent is not None:
            pub, kind = ent
            pub.publish(self.convert(kind, msg))
