"""Node shims around the device front-end that keep the reference's topics and message layouts
(SURVEY.md §8(f) row 1), plus an in-process runner that replays an npz dataset directory the
way `launch/*.launch` wires the nodes and writes the odometry as a TUM trajectory (row 2).

  PointCloudOdometryNode   scripts/PointCloudOdometry_noSeg.py:62-127
      per npz frame -> /velodyne_points (PointCloud2, xyz @ 0/4/8, step 12)
                    -> /frame_odom1    (Float64MultiArray data = [tx, ty, tz, qx, qy, qz, qw])
  FrameFeatureNode         src/frameFeature.cpp:35-139
      /velodyne_points -> /plane_frame_cloud1 (PointXYZI layout, stamp copied, frame "map")
                       -> /org_frame_cloud1   (the input, frame "map")
  LidarOdometryNode        src/lidarOdometry_onlyPC.cpp:85-124, 147-311  (run_onlyPC.launch)
      /plane_frame_cloud1 -> /frame_odom2 (Odometry, frame "map", child "map_child")
                          -> /frame_odom_path2 (Path of every pose so far)
                          -> /plane_frame_cloud2 (the current plane cloud, frame "map")
  LidarOdometryIngestNode  src/lidarOdometry.cpp:78-205  (run_noSeg / run_Seg launch graphs)
      /frame_odom1 -> odometryQueue;  /plane_frame_cloud1 -> pops the queue front from the
      second plane cloud on and accumulates it -> /frame_odom2, /frame_odom_path2,
      /plane_frame_cloud2 (no registration: the pose is the SSF Kabsch pose)

rospy, sensor_msgs and nav_msgs are not in this image: messages are the plain stand-ins of
`ssf.io` / below, and a `Bus` delivers them in-process.  Subscribed callbacks are duck-typed
(any object with the sensor_msgs/PointCloud2 attributes works), so wiring a node to rospy is
`rospy.Subscriber(topic, PointCloud2, node.on_cloud)` plus a publish callable that converts
the stand-in to the real message class.
"""
from __future__ import annotations

import copy
from collections import defaultdict, deque
from dataclasses import dataclass, field

import numpy as np
import torch

from . import io as sio
from ._abi import SSFError
from .frontend import Frontend, PlaneBatch, frame_offsets, identity_poses


@dataclass
class Float64MultiArray:
    data: list = field(default_factory=list)


@dataclass
class Pose:
    position: tuple = (0.0, 0.0, 0.0)
    orientation: tuple = (0.0, 0.0, 0.0, 1.0)      # x, y, z, w


@dataclass
class Odometry:
    header: sio.Header = field(default_factory=sio.Header)
    child_frame_id: str = ""
    pose: Pose = field(default_factory=Pose)


@dataclass
class Path:
    header: sio.Header = field(default_factory=sio.Header)
    poses: list = field(default_factory=list)      # (Header, Pose) pairs (geometry_msgs/PoseStamped)


class Bus:
    """In-process topic bus: publish(topic, msg) calls every subscriber in subscription order
    and keeps the last `keep` messages per topic."""

    def __init__(self, keep: int = 0):
        self.subs = defaultdict(list)
        self.keep = keep
        self.log = defaultdict(list)

    def subscribe(self, topic, cb):
        self.subs[topic].append(cb)

    def publish(self, topic, msg):
        if self.keep:
            lg = self.log[topic]
            lg.append(msg)
            del lg[:-self.keep]
        for cb in self.subs[topic]:
            cb(msg)


def _single_batch(xyzi: torch.Tensor, device) -> PlaneBatch:
    m = int(xyzi.shape[0])
    off, h_off = frame_offsets([m], device)
    return PlaneBatch(xyzi, torch.tensor([m], dtype=torch.int32, device=device), off, h_off, max(m, 1))


class FrameFeatureNode:
    """src/frameFeature.cpp cloudHandler on the device (k_bin_count / k_bin_scan / k_bin_curv / k_select)."""

    def __init__(self, publish, n_rows: int = 64, device=None, frontend: Frontend | None = None):
        self.fe = frontend or Frontend(n_rows, device=device)
        self.publish = publish

    def on_cloud(self, msg):
        view, ox = sio.cloud_points(msg)
        pts = torch.from_numpy(np.array(view, dtype=np.float32)).to(self.fe.device)  # msg bytes are read-only
        planes = self.fe.extract_planes(pts, xyz_offset=ox)                 # :45-123
        stamp = sio.stamp_of(msg.header)
        self.publish("/plane_frame_cloud1", sio.xyzi_to_cloud(planes, stamp, "map"))   # :129-133
        org = copy.copy(msg)                                                  # :135-138
        org.header = sio.Header(stamp[0], stamp[1], "map")
        self.publish("/org_frame_cloud1", org)
        return planes


class LidarOdometryNode:
    """src/lidarOdometry_onlyPC.cpp: the first plane cloud only becomes the last frame; every
    later one is registered against it (association, plane table, Ceres-style LM or GN) and the
    accumulated pose is published.  para_q/para_t (the warm start) and q_0_curr/t_0_curr stay on
    the device between frames."""

    def __init__(self, publish, n_rows: int = 64, device=None, solver: str = "ceres_lm",
                 max_iter: int | None = None, frontend: Frontend | None = None):
        self.fe = frontend or Frontend(n_rows, device=device, solver=solver, max_iter=max_iter)
        self.publish = publish
        dev = self.fe.device
        self.pose_rel = identity_poses(1, dev)      # para_q, para_t (:49-50)
        self.pose_abs = identity_poses(1, dev)      # q_0_last / t_0_last (:87-90)
        self.last = None
        self.last_table = None
        self.path = Path(sio.Header(0, 0, "map"))
        self.num_frame = 0

    def on_plane_cloud(self, msg):
        self.num_frame += 1
        xyzi = torch.from_numpy(sio.cloud_xyzi(msg)).to(self.fe.device)
        curr = _single_batch(xyzi, self.fe.device)
        table = self.fe.plane_table(curr)            # this frame's 30-NN planes, used next frame
        stamp = sio.stamp_of(msg.header)
        result = None
        if self.last is not None:                    # flagStart (:301-306)
            self.fe.register(self.last, self.last_table, curr, self.pose_rel, self.pose_abs)
            result = self._publish_result(stamp, xyzi)
        self.last, self.last_table = curr, table     # *lastFramePlanePtr = *currFramePlanePtr (:307)
        return result

    def _publish_result(self, stamp, xyzi):
        p = self.pose_abs[0].cpu().numpy()
        hdr = sio.Header(stamp[0], stamp[1], "map")
        pose = Pose(tuple(float(v) for v in p[4:7]), tuple(float(v) for v in p[0:4]))
        odom = Odometry(hdr, "map_child", pose)
        self.publish("/frame_odom2", odom)                                    # :98-109
        self.path.poses.append((hdr, pose))                                   # :111-118
        self.path.header = sio.Header(stamp[0], stamp[1], "map")
        self.publish("/frame_odom_path2", self.path)
        self.publish("/plane_frame_cloud2", sio.xyzi_to_cloud(xyzi, stamp, "map"))   # :120-124
        return odom


class LidarOdometryIngestNode:
    """src/lidarOdometry.cpp, the odometry node of the SSF launch graphs (run_noSeg.launch:8,
    run_Seg.launch:8): no registration -- the relative pose comes from /frame_odom1.

    odomHandler (:169-173) queues every /frame_odom1 message; cloudThread (:176-205) takes plane
    clouds in order, the first one only sets flagStart, and every later one pops the FRONT of the
    odometry queue (frameRegistration, :145-159: data[0:3] -> para_t, data[3:7] -> para_q x,y,z,w)
    and accumulates it (publishResult :80-83) on the device.  With the publisher's order (cloud
    first, then its pose) plane cloud k therefore consumes the pose published with frame k - 1.
    The reference reads front() of an EMPTY queue when a plane cloud overtakes the poses (UB,
    :148); here that raises SSFError."""

    def __init__(self, publish, device=None, frontend: Frontend | None = None):
        self.fe = frontend or Frontend(64, device=device)
        self.publish = publish
        self.queue = deque()                        # odometryQueue
        self.flag_start = False
        self.q_0_last = [0.0, 0.0, 0.0, 1.0]        # q_0_last / t_0_last (:68-71)
        self.t_0_last = [0.0, 0.0, 0.0]
        self.path = Path(sio.Header(0, 0, "map"))
        self.num_frame = 0

    def on_odom(self, msg):
        data = [float(v) for v in msg.data]
        if len(data) < 7:
            raise SSFError(f"/frame_odom1 carries {len(data)} values, expected [t(3), q(4)]")
        self.queue.append(data)

    def on_plane_cloud(self, msg):
        self.num_frame += 1
        stamp = sio.stamp_of(msg.header)
        if not self.flag_start:                     # :196-197
            self.flag_start = True
            return None
        if not self.queue:
            raise SSFError("plane cloud before its /frame_odom1 pose: the reference reads "
                           "odometryQueue.front() of an empty queue here (lidarOdometry.cpp:148)")
        d = self.queue.popleft()                    # frameRegistration (:147-155)
        rel = torch.tensor([[d[3], d[4], d[5], d[6], d[0], d[1], d[2]]], dtype=torch.float64,
                           device=self.fe.device)
        start = self.q_0_last + self.t_0_last
        ab = self.fe.accumulate_sequence(rel, start=start)[0].cpu().numpy()   # :80-83
        self.q_0_last = [float(v) for v in ab[0:4]]
        self.t_0_last = [float(v) for v in ab[4:7]]
        hdr = sio.Header(stamp[0], stamp[1], "map")
        pose = Pose(tuple(self.t_0_last), tuple(self.q_0_last))
        odom = Odometry(hdr, "map_child", pose)
        self.publish("/frame_odom2", odom)                                    # :96-107
        self.path.poses.append((hdr, pose))                                   # :109-116
        self.path.header = sio.Header(stamp[0], stamp[1], "map")
        self.publish("/frame_odom_path2", self.path)
        xyzi = sio.cloud_xyzi(msg)                                            # :118-122
        self.publish("/plane_frame_cloud2", sio.xyzi_to_cloud(xyzi, stamp, "map"))
        return odom


class PointCloudOdometryNode:
    """The data-source node of the launch graphs, for one npz frame: publish the cloud, then
      mode 'gmm'  -- PointCloudOdometry_noSeg.py:62-127: GMM mask + Kabsch pose as [t, q];
      mode 'gt'   -- PointCloudOdometry.py:60-105: background = s_fg_mask == 0, Kabsch, [t, q];
      mode 'none' -- PointCloudOdometry_onlyPC.py:37-65: the cloud only (no /frame_odom1)."""

    def __init__(self, publish, device=None, frontend: Frontend | None = None, mode: str = "gmm",
                 seed: int | None = None):
        if mode not in ("gmm", "gt", "none"):
            raise ValueError(f"mode {mode!r}")
        self.fe = frontend or Frontend(64, device=device)
        self.publish = publish
        self.mode = mode
        if seed is not None:
            self.fe.seed(seed)

    def on_frame(self, pos1, flow=None, stamp=(0, 0), gt_mask=None):
        dev = self.fe.device
        pos = pos1 if isinstance(pos1, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(pos1, np.float32))
        pos = pos.to(dev, torch.float32).contiguous()
        self.publish("/velodyne_points", sio.xyz_to_cloud(pos.cpu().numpy(), stamp, "livox_frame"))   # :73-94
        if self.mode == "none":
            return None
        fl = flow if isinstance(flow, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(flow, np.float32))
        fl = fl.to(dev, torch.float32).contiguous()
        off, h_off = frame_offsets([pos.shape[0]], dev)
        m = None
        if self.mode != "gmm":
            m = torch.as_tensor(np.asarray(gt_mask) if not isinstance(gt_mask, torch.Tensor) else gt_mask)
            m = m.to(dev, torch.uint8).contiguous()
        out, _ = self.fe.mask_pose(pos, fl, off, h_off, mode=self.mode, mask_in=m, want_mask=False)
        o = out[0].cpu().numpy()
        msg = Float64MultiArray([float(v) for v in o[0:7]])                   # hstack((t, q)) :123-125
        self.publish("/frame_odom1", msg)
        return o


class MapOptimizationNode:
    """src/mapOptmization.cpp cloudThread/mapOptimization (:429-467) for one sequence: pairs
    /plane_frame_cloud2 with /frame_odom2 (stamps within 5 ms, :434-439), keeps keyframes,
    detects loops and registers them on the GPU (ssf.loop.LoopCloser), publishes
    /map_odom_res3 (Odometry "map" / "map_child"), /map_frame_res3 (the frame in the map) and
    /map_laser_path_res3, and appends TUM lines to RESULT_PATH (:355-374).  GTSAM iSAM2 is not
    part of this path: the published pose is the loop-adjusted odometry trans_loop_adjust *
    T_fodom_0_curr (:450) at every frame (the reference publishes its iSAM2 estimate for
    keyframes only), and the loop constraints are kept in ``closer.constraints``."""

    def __init__(self, publish, device=None, frontend: Frontend | None = None,
                 tum_path: str | None = None):
        from .loop import LoopCloser, get_translation_and_euler_angles  # noqa: F401
        self.publish = publish
        self.fe = frontend or Frontend(64, device=device)
        self.closer = LoopCloser(self.fe)
        self.planes, self.odoms = [], []          # planeQueue / odometryQueue (:65-75)
        self.path = Path()
        self.writer = sio.TumWriter(tum_path) if tum_path else None

    def on_plane_cloud(self, msg):
        self.planes.append(msg)
        self._drain()

    def on_odom(self, msg):
        self.odoms.append(msg)
        self._drain()

    def _drain(self):
        import numpy as np
        from .loop import transform_cloud
        from scipy.spatial.transform import Rotation
        while self.planes and self.odoms:
            pm, om = self.planes[0], self.odoms[0]
            tp, to = sio.stamp_of(pm.header), sio.stamp_of(om.header)
            if abs((tp[0] - to[0]) + (tp[1] - to[1]) * 1e-9) > 0.005:    # time sync (:436-439)
                return
            self.planes.pop(0)
            self.odoms.pop(0)
            xyzi = torch.from_numpy(sio.cloud_xyzi(pm)).to(self.fe.device)
            stamp = tp[0] + tp[1] * 1e-9
            T, _, _ = self.closer.process(xyzi, om.pose.orientation, om.pose.position, stamp)
            q = Rotation.from_matrix(T[:3, :3]).as_quat()                  # x, y, z, w
            hdr = sio.Header(tp[0], tp[1], "map")
            pose = Pose(tuple(float(v) for v in T[:3, 3]), tuple(float(v) for v in q))
            self.publish("/map_odom_res3", Odometry(hdr, "map_child", pose))
            if self.writer:
                self.writer.write(tp, pose.position, pose.orientation)
            self.path.poses.append((hdr, pose))
            self.path.header = hdr
            self.publish("/map_laser_path_res3", self.path)
            self.publish("/map_frame_res3", sio.xyzi_to_cloud(transform_cloud(xyzi, T), tp, "map"))


LAUNCH_GRAPHS = {
    # launch file: (data-source mode, odometry node, npz keys)
    "onlyPC": ("none", "registration", ("pos1",)),             # run_onlyPC.launch:7-15
    "noSeg": ("gmm", "ingest", ("pos1", "gt")),                 # run_noSeg.launch:7-16
    "Seg": ("gt", "ingest", ("pos1", "gt", "s_fg_mask")),       # run_Seg.launch:7-16
}


def run_sequence(root: str, tum_path: str | None = None, n_rows: int = 64, device=None,
                 solver: str = "ceres_lm", max_iter: int | None = None, seed: int | None = None,
                 rate_hz: float = 10.0, launch: str = "onlyPC", map_tum_path: str | None = None,
                 truncate_results: bool = False):
    """Replay a DATASET_PATH directory through the node graph of launch/run_<launch>.launch:
      onlyPC: PointCloudOdometry_onlyPC -> frameFeature -> lidarOdometry_onlyPC (registration)
      noSeg:  PointCloudOdometry_noSeg (GMM mask + Kabsch -> /frame_odom1) -> frameFeature ->
              lidarOdometry (pose ingest + accumulation)
      Seg:    PointCloudOdometry (ground-truth mask s_fg_mask == 0) -> same as noSeg
    plus mapOptmization when `map_tum_path` is given.  Stamps are synthetic and monotone (frame k
    at k / rate_hz; the reference uses wall-clock ros::Time::now()).  The /frame_odom2 poses are
    appended to `tum_path` as TUM lines (like the reference, an existing file is extended unless
    truncate_results=True).
    -> dict(odom1 [F, 7] f64 [t, q] (empty for onlyPC), odom2 [F-1, 7] f64 [t, q], stamps)"""
    if launch not in LAUNCH_GRAPHS:
        raise ValueError(f"launch {launch!r}: one of {sorted(LAUNCH_GRAPHS)}")
    src_mode, odo_kind, keys = LAUNCH_GRAPHS[launch]
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    bus = Bus()
    pco = PointCloudOdometryNode(bus.publish, device=dev, seed=seed, mode=src_mode)
    ff = FrameFeatureNode(bus.publish, n_rows=n_rows, device=dev)
    if odo_kind == "registration":
        lo = LidarOdometryNode(bus.publish, n_rows=n_rows, device=dev, solver=solver, max_iter=max_iter)
    else:
        lo = LidarOdometryIngestNode(bus.publish, device=dev)
        bus.subscribe("/frame_odom1", lo.on_odom)
    bus.subscribe("/velodyne_points", ff.on_cloud)
    bus.subscribe("/plane_frame_cloud1", lo.on_plane_cloud)
    odom1, odom2, stamps = [], [], []
    if tum_path and truncate_results:
        open(tum_path, "w").close()
    writer = sio.TumWriter(tum_path) if tum_path else None

    def on_odom1(msg):
        odom1.append(list(msg.data))

    def on_odom2(msg):
        odom2.append(list(msg.pose.position) + list(msg.pose.orientation))
        if writer:
            writer.write((msg.header.stamp_sec, msg.header.stamp_nsec), msg.pose.position,
                         msg.pose.orientation)

    bus.subscribe("/frame_odom1", on_odom1)
    bus.subscribe("/frame_odom2", on_odom2)
    mo = None
    if map_tum_path is not None:                     # mapOptmization on /plane_frame_cloud2 + /frame_odom2
        if map_tum_path and truncate_results:
            open(map_tum_path, "w").close()
        mo = MapOptimizationNode(bus.publish, device=dev, tum_path=map_tum_path or None)
        bus.subscribe("/plane_frame_cloud2", mo.on_plane_cloud)
        bus.subscribe("/frame_odom2", mo.on_odom)
    period_ns = int(round(1e9 / rate_hz))
    for fr in sio.NpzSequence(root, keys=keys, device=dev):
        t_ns = fr["index"] * period_ns
        stamp = (t_ns // 1_000_000_000, t_ns % 1_000_000_000)
        stamps.append(stamp)
        pco.on_frame(fr["pos1"], fr.get("gt"), stamp,
                     gt_mask=fr.get("s_fg_mask") if src_mode == "gt" else None)
    return dict(odom1=np.asarray(odom1, np.float64).reshape(-1, 7),
                odom2=np.asarray(odom2, np.float64).reshape(-1, 7), stamps=stamps,
                loops=mo.closer.constraints if mo else [])
