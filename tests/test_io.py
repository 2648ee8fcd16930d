"""Caller-side formats: PointCloud2 layouts of the reference's topics,
the npz sequence file list, and the TUM writer's text format.  CPU only."""
import os

import numpy as np
import pytest

from ssf import io as sio


def test_velodyne_layout_roundtrip():
    rng = np.random.default_rng(0)
    pts = rng.normal(size=(1000, 3)).astype(np.float32)
    msg = sio.xyz_to_cloud(pts, stamp=(12, 5), frame_id="livox_frame")
    # PointCloudOdometry_noSeg.py:73-92: fields x/y/z FLOAT32 at 0/4/8, point_step 12
    assert [(f.name, f.offset, f.datatype, f.count) for f in msg.fields] == \
        [("x", 0, 7, 1), ("y", 4, 7, 1), ("z", 8, 7, 1)]
    assert msg.point_step == 12 and msg.row_step == 12000 and msg.height == 1 and msg.width == 1000
    assert not msg.is_bigendian and not msg.is_dense
    assert msg.data == pts.tobytes()
    assert np.array_equal(sio.cloud_xyz(msg), pts)
    view, ox = sio.cloud_points(msg)
    assert ox == 0 and view.shape == (1000, 3)


def test_asf_malformed_intensity_is_ignored():
    """main_sju_occ_ros.py:243-249 declares intensity at offset 12 with point_step 12 (SURVEY
    A.1): only x, y, z are read."""
    pts = np.arange(30, dtype=np.float32).reshape(10, 3)
    msg = sio.xyz_to_cloud(pts)
    msg.fields = list(msg.fields) + [sio.PointField("intensity", 12)]
    assert np.array_equal(sio.cloud_xyz(msg), pts)
    with pytest.raises(sio.SSFError):
        sio.cloud_xyzi(msg)          # the intensity field lies outside the 12-byte point


def test_xyzi_plane_cloud_layout():
    """pcl::toROSMsg(PointCloud<PointXYZI>): 32-byte points, intensity at 16."""
    rng = np.random.default_rng(1)
    a = rng.normal(size=(57, 4)).astype(np.float32)
    msg = sio.xyzi_to_cloud(a, stamp=(3, 999999999))
    assert msg.point_step == 32 and msg.row_step == 32 * 57 and msg.is_dense
    assert [(f.name, f.offset) for f in msg.fields] == [("x", 0), ("y", 4), ("z", 8), ("intensity", 16)]
    raw = np.frombuffer(msg.data, np.float32).reshape(57, 8)
    assert np.all(raw[:, 3] == 0) and np.all(raw[:, 5:] == 0)
    assert np.array_equal(sio.cloud_xyzi(msg), a)
    assert sio.stamp_of(msg.header) == (3, 999999999)


def test_strided_cloud_with_offset_xyz():
    """A generic driver layout (ring/time words before x) is read through the field offsets."""
    n = 20
    rec = np.zeros((n, 6), np.float32)
    rec[:, 2:5] = np.arange(3 * n, dtype=np.float32).reshape(n, 3)
    msg = sio.PointCloud2(sio.Header(), 1, n, [sio.PointField("x", 8), sio.PointField("y", 12),
                                                 sio.PointField("z", 16)], False, 24, 24 * n,
                          rec.tobytes(), True)
    view, ox = sio.cloud_points(msg)
    assert ox == 8 and view.shape == (n, 6)
    assert np.array_equal(sio.cloud_xyz(msg), rec[:, 2:5])


@pytest.mark.parametrize("bad", ["big", "short", "nonconsec", "f64"])
def test_bad_layouts_raise(bad):
    msg = sio.xyz_to_cloud(np.zeros((4, 3), np.float32))
    if bad == "big":
        msg.is_bigendian = True
    elif bad == "short":
        msg.data = msg.data[:-4]
    elif bad == "nonconsec":
        msg.fields = [sio.PointField("x", 0), sio.PointField("z", 4), sio.PointField("y", 8)]
    else:
        msg.fields = [sio.PointField("x", 0, sio.FLOAT64), sio.PointField("y", 4), sio.PointField("z", 8)]
    with pytest.raises(sio.SSFError):
        sio.cloud_xyz(msg)


def test_tum_line_matches_cpp_stream_format():
    """std::fixed, precision 6 for the pose; ros::Time prints sec.nsec (9 digits)."""
    line = sio.tum_line((1700000000, 5000), [1.0, -0.0, 2.5e-7], [0.0, 0.0, 0.70710678118, 0.70710678118])
    assert line == "1700000000.000005000 1.000000 -0.000000 0.000000 0.000000 0.000000 0.707107 0.707107"
    assert sio.tum_line("7.5", [1234.5678915, 0, 0], [0, 0, 0, 1]).startswith("7.5 1234.567892 ")


def test_tum_writer_roundtrip(tmp_path):
    p = str(tmp_path / "traj.txt")
    w = sio.TumWriter(p)
    poses = np.array([[0, 0, 0, 1, 0, 0, 0], [0, 0, 0.1, 0.995, 1.25, -0.5, 0.01]])
    w.write_poses([(1, 0), (1, 100000000)], poses)
    w.write((2, 0), [3.0, 4.0, 5.0], [0, 0, 0, 1])
    stamps, t, q = sio.read_tum(p)
    assert stamps == ["1.000000000", "1.100000000", "2.000000000"]
    assert np.allclose(t[1], [1.25, -0.5, 0.01]) and np.allclose(q[1], [0, 0, 0.1, 0.995])
    assert open(p).read().count("\n") == 3


def test_sequence_files_order_and_safe_load(tmp_path):
    """sorted(listdir) + glob + sort (PointCloudOdometry_noSeg.py:54-60); npz read without
    unpickling: an object array is refused."""
    for name in ["0010.npz", "0002.npz", "0001.npz"]:
        np.savez(str(tmp_path / name), pos1=np.ones((5, 3), np.float64), gt=np.zeros((5, 3)))
    files = sio.sequence_files(str(tmp_path))
    assert [os.path.basename(f) for f in files] == ["0001.npz", "0002.npz", "0010.npz"]
    fr = sio.load_frame(files[0])
    assert fr["pos1"].dtype == np.float32 and fr["pos1"].shape == (5, 3)
    np.savez(str(tmp_path / "0003.npz"), pos1=np.array([{"a": 1}], dtype=object), gt=np.zeros((1, 3)))
    with pytest.raises(ValueError):
        sio.load_frame(str(tmp_path / "0003.npz"))
    with pytest.raises(sio.SSFError):
        sio.load_frame(files[0], keys=("pos1", "flow"))


def test_tum_writer_appends_like_the_reference(tmp_path):
    """mapOptmization.cpp:355 opens RESULT_PATH with std::ios::app only: an existing
    trajectory is extended, never wiped (truncation is an explicit runner option)."""
    p = str(tmp_path / "traj.txt")
    with open(p, "w") as f:
        f.write("0.000000000 0 0 0 0 0 0 1\n")
    sio.TumWriter(p).write((1, 0), [1.0, 2.0, 3.0], [0, 0, 0, 1])
    assert open(p).read().count("\n") == 2
    sio.TumWriter(p, truncate=True).write((2, 0), [1.0, 2.0, 3.0], [0, 0, 0, 1])
    assert open(p).read().count("\n") == 1


def test_organized_cloud_with_padded_rows():
    """height > 1 with row_step > width * point_step: each row is read at its row_step."""
    h, w, step, pad = 3, 5, 16, 24
    rows = np.zeros((h, w * step + pad), np.uint8)
    pts = np.arange(h * w * 3, dtype=np.float32).reshape(h, w, 3)
    for r in range(h):
        rec = np.zeros((w, 4), np.float32)
        rec[:, :3] = pts[r]
        rows[r, : w * step] = rec.view(np.uint8).reshape(-1)
        rows[r, w * step:] = 0xFF                      # padding garbage must not leak in
    msg = sio.PointCloud2(sio.Header(), h, w, list(sio.VELODYNE_FIELDS), False, step,
                          w * step + pad, rows.tobytes(), True)
    assert np.array_equal(sio.cloud_xyz(msg), pts.reshape(-1, 3))
    msg.row_step = w * step - 4
    with pytest.raises(sio.SSFError):
        sio.cloud_xyz(msg)
    msg.row_step = w * step + pad
    msg.data = msg.data[:-(pad + 4)]
    with pytest.raises(sio.SSFError):
        sio.cloud_xyz(msg)
