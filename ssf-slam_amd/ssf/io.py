"""Caller-side data formats of the front-end.

* PointCloud2 ingest / egress, with the reference's topic layouts:
  - `/velodyne_points`: x, y, z FLOAT32 at byte offsets 0/4/8, point_step 12, height 1, little
    endian (`scripts/PointCloudOdometry_noSeg.py:73-92`).  Extra fields (the ASF nodes' malformed
    `intensity` at offset 12 with point_step 12, `main_sju_occ_ros.py:243-249`) are ignored, as
    SURVEY Appendix A.1 prescribes.
  - `/plane_frame_cloud1/2`: `pcl::toROSMsg` of a `pcl::PointCloud<PointXYZI>`: x, y, z,
    intensity FLOAT32 at 0/4/8/16, point_step 32 (`src/frameFeature.cpp:129-133`,
    `src/lidarOdometry_onlyPC.cpp:120-124`).
* The npz sequence loader of `PointCloudOdometry_noSeg.py:54-68` (sorted file list, `pos1` and
  `gt` = flow), read with `np.load(allow_pickle=False)`.  Frames are staged in pinned host
  memory by a reader thread and copied to the device on a side stream one frame ahead, so file
  IO and PCIe overlap the kernels of the current frame.
* The TUM trajectory writer of `src/mapOptmization.cpp:355-374`: `stamp x y z qx qy qz qw`,
  `std::fixed` with precision 6; the stamp goes through `ros::Time`'s `operator<<` (sec.nsec,
  nsec zero-padded to 9 digits) and is unaffected by the precision.

Messages are duck-typed: anything with the sensor_msgs/PointCloud2 attributes (a real rospy
message included) is accepted; `PointCloud2` below is the plain stand-in used when rospy is
absent (it is absent in this image).
"""
from __future__ import annotations

import glob
import os
import queue
import threading
from dataclasses import dataclass, field

import numpy as np
import torch

from ._abi import SSFError

# sensor_msgs/PointField datatypes
INT8, UINT8, INT16, UINT16, INT32, UINT32, FLOAT32, FLOAT64 = range(1, 9)


@dataclass
class PointField:
    name: str
    offset: int
    datatype: int = FLOAT32
    count: int = 1


@dataclass
class Header:
    stamp_sec: int = 0
    stamp_nsec: int = 0
    frame_id: str = ""

    @property
    def stamp(self) -> float:          # ros::Time::toSec()
        return self.stamp_sec + 1e-9 * self.stamp_nsec


@dataclass
class PointCloud2:
    header: Header = field(default_factory=Header)
    height: int = 1
    width: int = 0
    fields: list = field(default_factory=list)
    is_bigendian: bool = False
    point_step: int = 0
    row_step: int = 0
    data: bytes = b""
    is_dense: bool = False


VELODYNE_FIELDS = (PointField("x", 0), PointField("y", 4), PointField("z", 8))
XYZI_FIELDS = (PointField("x", 0), PointField("y", 4), PointField("z", 8), PointField("intensity", 16))
XYZI_STEP = 32


def stamp_of(header) -> tuple:
    """(sec, nsec) of a Header stand-in or of a rospy std_msgs/Header."""
    if hasattr(header, "stamp_sec"):
        return int(header.stamp_sec), int(header.stamp_nsec)
    st = header.stamp
    return int(st.secs), int(st.nsecs)


def _field_offsets(msg, names):
    by = {f.name: f for f in msg.fields}
    out = []
    for nm in names:
        f = by.get(nm)
        if f is None:
            raise SSFError(f"PointCloud2 has no '{nm}' field")
        if f.datatype != FLOAT32 or f.count != 1:
            raise SSFError(f"PointCloud2 field '{nm}' must be one FLOAT32")
        out.append(int(f.offset))
    return out


def cloud_points(msg):
    """PointCloud2 -> (host array [n, point_step/4] f32 of its points, byte offset of x).  x, y, z
    must be consecutive FLOAT32s, which every layout the reference publishes satisfies.  An
    organized cloud (height > 1) is read row by row at `row_step`, so padded rows are skipped
    (row_step 0, as some publishers leave it, means dense rows)."""
    if msg.is_bigendian:
        raise SSFError("big-endian PointCloud2 is not supported")
    ox, oy, oz = _field_offsets(msg, ("x", "y", "z"))
    if oy != ox + 4 or oz != ox + 8 or ox % 4:
        raise SSFError("x, y, z must be consecutive, 4-byte aligned FLOAT32 fields")
    step = int(msg.point_step)
    n = int(msg.width) * int(msg.height)
    if step % 4 or step < ox + 12:
        raise SSFError(f"unsupported point_step {step}")
    w, h = int(msg.width), int(msg.height)
    row_step = int(getattr(msg, "row_step", 0) or 0) or w * step
    if row_step < w * step or row_step % 4:
        raise SSFError(f"row_step {row_step} shorter than width * point_step or unaligned")
    if n == 0:
        return np.zeros((0, step // 4), np.float32), ox
    if (h - 1) * row_step + w * step > len(msg.data):
        raise SSFError("PointCloud2 data shorter than its rows (height * row_step)")
    if row_step == w * step:
        buf = np.frombuffer(msg.data, dtype="<f4", count=n * step // 4)
        return buf.reshape(n, step // 4), ox
    rows = np.frombuffer(msg.data, dtype=np.uint8, count=(h - 1) * row_step + w * step)
    out = np.empty((h, w * step), np.uint8)
    for r in range(h):
        out[r] = rows[r * row_step:r * row_step + w * step]
    return out.view("<f4").reshape(n, step // 4), ox


def cloud_xyz(msg) -> np.ndarray:
    """PointCloud2 -> contiguous [n, 3] f32 (pcl::fromROSMsg into PointXYZ)."""
    pts, ox = cloud_points(msg)
    k = ox // 4
    return np.ascontiguousarray(pts[:, k:k + 3])


def cloud_xyzi(msg) -> np.ndarray:
    """PointCloud2 with an `intensity` field -> [n, 4] f32 x, y, z, intensity."""
    pts, ox = cloud_points(msg)
    (oi,) = _field_offsets(msg, ("intensity",))
    if oi % 4 or oi + 4 > int(msg.point_step):
        raise SSFError("intensity field outside the point or unaligned")
    k = ox // 4
    out = np.empty((pts.shape[0], 4), np.float32)
    out[:, :3] = pts[:, k:k + 3]
    out[:, 3] = pts[:, oi // 4]
    return out


def xyz_to_cloud(points, stamp=(0, 0), frame_id="livox_frame") -> PointCloud2:
    """[n, 3] -> the `/velodyne_points` layout (PointCloudOdometry_noSeg.py:73-92)."""
    p = np.ascontiguousarray(np.asarray(points, np.float32).reshape(-1, 3))
    return PointCloud2(Header(int(stamp[0]), int(stamp[1]), frame_id), 1, p.shape[0],
                       list(VELODYNE_FIELDS), False, 12, 12 * p.shape[0], p.tobytes(), False)


def xyzi_to_cloud(xyzi, stamp=(0, 0), frame_id="map") -> PointCloud2:
    """[m, 4] x, y, z, intensity (a plane cloud) -> the pcl::toROSMsg(PointXYZI) layout: 32-byte
    points, intensity at offset 16, padding words zero, is_dense true as pcl sets it."""
    a = xyzi.detach().cpu().numpy() if isinstance(xyzi, torch.Tensor) else np.asarray(xyzi)
    a = a.astype(np.float32, copy=False).reshape(-1, 4)
    m = a.shape[0]
    rec = np.zeros((m, XYZI_STEP // 4), np.float32)
    rec[:, 0:3] = a[:, 0:3]
    rec[:, 4] = a[:, 3]
    return PointCloud2(Header(int(stamp[0]), int(stamp[1]), frame_id), 1, m, list(XYZI_FIELDS), False,
                       XYZI_STEP, XYZI_STEP * m, rec.tobytes(), True)


# ---------------------------------------------------------------------------- npz sequences
def sequence_files(root: str) -> list:
    """The reference's file list: every entry of sorted(os.listdir(root)) globbed, then sorted
    (PointCloudOdometry_noSeg.py:54-60)."""
    files = []
    for sub in sorted(os.listdir(root)):
        files += glob.glob(os.path.join(root, sub))
    files.sort()
    return files


def load_frame(path: str, keys=("pos1", "gt")) -> dict:
    """One npz frame as contiguous f32 arrays; never unpickles (allow_pickle=False)."""
    with np.load(path, allow_pickle=False) as z:
        missing = [k for k in keys if k not in z.files]
        if missing:
            raise SSFError(f"{path}: missing arrays {missing}")
        return {k: np.ascontiguousarray(z[k], dtype=np.float32) for k in keys}


class NpzSequence:
    """A DATASET_PATH directory of npz frames, iterated as device tensors.

    A reader thread loads up to `depth` frames ahead into pinned host buffers; the H2D copy of a
    frame runs on a dedicated stream and the consumer's current stream waits on its event, so
    file IO and the copy overlap the kernels of the previous frame."""

    def __init__(self, root: str, keys=("pos1", "gt"), device=None, depth: int = 2):
        self.files = sequence_files(root)
        self.keys = tuple(keys)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.depth = max(1, int(depth))

    def __len__(self):
        return len(self.files)

    def host(self, i: int) -> dict:
        return load_frame(self.files[i], self.keys)

    def __iter__(self):
        q: queue.Queue = queue.Queue(maxsize=self.depth)
        stop = threading.Event()

        def put(item):
            while not stop.is_set():
                try:
                    q.put(item, timeout=0.1)
                    return True
                except queue.Full:
                    continue
            return False

        def reader():
            try:
                for i, f in enumerate(self.files):
                    fr = load_frame(f, self.keys)
                    pinned = {k: torch.from_numpy(v).pin_memory() for k, v in fr.items()}
                    if not put((i, f, pinned)):
                        return
                put(None)
            except BaseException as e:          # surfaced in the consumer
                put(e)

        th = threading.Thread(target=reader, daemon=True)
        th.start()
        copy_stream = torch.cuda.Stream(device=self.device)
        try:
            while True:
                item = q.get()
                if item is None:
                    return
                if isinstance(item, BaseException):
                    raise item
                i, f, pinned = item
                with torch.cuda.stream(copy_stream):
                    dev = {k: v.to(self.device, non_blocking=True) for k, v in pinned.items()}
                ev = torch.cuda.Event()
                ev.record(copy_stream)
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                for v in dev.values():
                    v.record_stream(cur)
                dev["index"] = i
                dev["path"] = f
                yield dev
        finally:
            stop.set()
            th.join(timeout=5.0)


# ---------------------------------------------------------------------------- TUM trajectory
def ros_time_str(sec: int, nsec: int) -> str:
    """ros::Time operator<<: sec '.' nsec as 9 zero-padded digits."""
    return f"{int(sec)}.{int(nsec):09d}"


def tum_line(stamp, t, q_xyzw) -> str:
    """`stamp x y z qx qy qz qw` as mapOptmization.cpp:362-372 writes it (std::fixed,
    precision 6).  `stamp` is (sec, nsec) or an already formatted string."""
    st = stamp if isinstance(stamp, str) else ros_time_str(*stamp)
    vals = [float(v) for v in t] + [float(v) for v in q_xyzw]
    return st + " " + " ".join(f"{v:.6f}" for v in vals)


class TumWriter:
    """Appends one line per pose to RESULT_PATH, reopening the file in append mode for every
    pose as the reference does (a crash loses at most the pose being written).  Like the
    reference (mapOptmization.cpp:355, std::ios::app only) an existing file is never wiped
    unless the runner asks for it explicitly (truncate=True)."""

    def __init__(self, path: str, truncate: bool = False):
        self.path = path
        if truncate:
            open(path, "w").close()

    def write(self, stamp, t, q_xyzw):
        with open(self.path, "a") as f:
            f.write(tum_line(stamp, t, q_xyzw) + "\n")

    def write_poses(self, stamps, poses):
        """poses [n, 7] (q xyzw, t), the layout of the device pose records."""
        p = poses.detach().cpu().numpy() if isinstance(poses, torch.Tensor) else np.asarray(poses)
        with open(self.path, "a") as f:
            for st, row in zip(stamps, p):
                f.write(tum_line(st, row[4:7], row[0:4]) + "\n")


def read_tum(path: str) -> tuple:
    """-> (stamps [n] str, t [n, 3], q_xyzw [n, 4]) of a TUM file."""
    stamps, vals = [], []
    with open(path) as f:
        for line in f:
            parts = line.split()
            if len(parts) != 8:
                continue
            stamps.append(parts[0])
            vals.append([float(v) for v in parts[1:]])
    a = np.asarray(vals, np.float64).reshape(-1, 7)
    return stamps, a[:, 0:3], a[:, 3:7]
