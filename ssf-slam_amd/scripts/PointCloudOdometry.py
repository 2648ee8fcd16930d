#!/usr/bin/env python3
"""Drop-in for the reference's scripts/PointCloudOdometry.py (a launch/*.launch `type=` target):
the same node, topics and ~DATASET_PATH parameter, with the mask / Kabsch block on the MI355X
front-end (ssf.entry.pointcloud_odometry_main).  Without rospy: --dataset PATH replays the launch
graph offline."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from ssf.entry import pointcloud_odometry_main  # noqa: E402

if __name__ == "__main__":
    pointcloud_odometry_main("PointCloudOdometry.py")
