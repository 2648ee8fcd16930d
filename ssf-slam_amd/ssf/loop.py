"""Loop-closure registration of mapOptmization (src/mapOptmization.cpp).

GPU work goes through the C ABI (loop.hip): ``voxel_grid`` <- pcl::VoxelGrid<PointXYZI>::filter
(downSizeFilterICP 0.1 m :214-217, downSizeFilterMap 0.4 m :406-409) and ``icp`` <-
pcl::IterativeClosestPoint<PointXYZI, PointXYZI> (:224-238).  ``LoopCloser`` mirrors the
keyframe / loop-detection / local-map logic around them (isKeyFrame :129-144,
addPose3D6D :78-107, detectLoopFrameID :167-197, getLoopLocalMap :200-218, addLoopFactor
:221-272, trans_loop_adjust :325, the T_map_0_curr chain :447-450) and emits the loop
constraint the reference adds to its GTSAM graph (BetweenFactor poseFrom.between(poseTo),
noise = the ICP fitness score).  GTSAM iSAM2 is not part of this path (absent from the image):
the published pose is the loop-adjusted odometry, see DESIGN.md.

Pose helpers restate pcl/common/eigen.h: getTransformation (roll/pitch/yaw -> affine,
yaw * pitch * roll) and getTranslationAndEulerAngles.  Key poses are stored in float, as the
reference's PointXYZIRPYT cloud holds them.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _abi
from .frontend import Frontend, _ptr, _stream


# --------------------------------------------------------------------------- pose helpers
def get_transformation(x, y, z, roll, pitch, yaw):
    """pcl::getTransformation (pcl/common/impl/eigen.hpp) in double -> 4x4."""
    A, B = math.cos(yaw), math.sin(yaw)
    Cc, D = math.cos(pitch), math.sin(pitch)
    E, F = math.cos(roll), math.sin(roll)
    DE, DF = D * E, D * F
    return np.array([[A * Cc, A * DF - B * E, B * F + A * DE, x],
                     [B * Cc, A * E + B * DF, B * DE - A * F, y],
                     [-D, Cc * F, Cc * E, z],
                     [0.0, 0.0, 0.0, 1.0]], np.float64)


def get_translation_and_euler_angles(t):
    """pcl::getTranslationAndEulerAngles -> (x, y, z, roll, pitch, yaw)."""
    return (float(t[0, 3]), float(t[1, 3]), float(t[2, 3]), math.atan2(t[2, 1], t[2, 2]),
            math.asin(-t[2, 0]), math.atan2(t[1, 0], t[0, 0]))


def pose_from_quat(q_xyzw, t):
    """Eigen::Affine3d: rotate(q) then pretranslate(t) (mapOptmization.cpp:447-449)."""
    x, y, z, w = (float(v) for v in q_xyzw)
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = np.asarray(t, np.float64)
    return T


def between(a, b):
    """gtsam Pose3 a.between(b) = a^-1 b (4x4)."""
    return np.linalg.inv(a) @ b


# --------------------------------------------------------------------------- GPU entry points
def voxel_grid(fe: Frontend, xyzi: torch.Tensor, off: torch.Tensor, h_off: torch.Tensor, leaf: float):
    """Batched pcl::VoxelGrid: float4 clouds at offsets -> (centroids at the same offsets,
    per-cloud counts (device int32))."""
    F = int(h_off.numel()) - 1
    out = torch.empty_like(xyzi)
    cnt = torch.zeros(max(F, 0), dtype=torch.int32, device=xyzi.device)
    ho = h_off.contiguous()
    fe._check(_abi.lib().ssf_voxel_grid_batch(fe._h, _stream(fe.device), F, _ptr(xyzi), _ptr(off),
                                              C.c_void_p(ho.data_ptr()), float(leaf), _ptr(out), _ptr(cnt)),
              "ssf_voxel_grid_batch")
    return out, cnt


def voxel_grid_one(fe: Frontend, xyzi: torch.Tensor, leaf: float) -> torch.Tensor:
    """One cloud through the batched filter (the mapOptmization call shape)."""
    n = int(xyzi.shape[0])
    h = torch.tensor([0, n], dtype=torch.int64)
    out, cnt = voxel_grid(fe, xyzi.contiguous(), h.to(xyzi.device), h, leaf)
    return out[: int(cnt[0])]


def icp_params(max_iter=100, max_corr_dist=50.0, trans_eps=1e-6, fit_eps=1e-6):
    p = _abi.IcpParams()
    _abi.lib().ssf_icp_params_default(C.byref(p))
    p.max_iter, p.max_corr_dist, p.trans_eps, p.fit_eps = int(max_iter), float(max_corr_dist), float(trans_eps), float(fit_eps)
    return p


def icp_batch(fe: Frontend, src, src_off, h_src_off, tgt, tgt_off, h_tgt_off, params=None, guess=None):
    """Batched ICP -> list of dicts (T 4x4 float32, fitness, converged, iterations, state, n_corr)."""
    P = int(h_src_off.numel()) - 1
    params = params or icp_params()
    out = np.zeros(P * _abi.ICP_OUT_STRIDE, np.float64)
    g = None if guess is None else np.ascontiguousarray(guess, np.float32).reshape(-1)
    hs, ht = h_src_off.contiguous(), h_tgt_off.contiguous()
    fe._check(_abi.lib().ssf_icp_batch(fe._h, _stream(fe.device), P, _ptr(src), _ptr(src_off),
                                       C.c_void_p(hs.data_ptr()), _ptr(tgt), _ptr(tgt_off),
                                       C.c_void_p(ht.data_ptr()), C.byref(params),
                                       None if g is None else g.ctypes.data_as(C.c_void_p),
                                       out.ctypes.data_as(C.c_void_p)), "ssf_icp_batch")
    res = []
    for k in range(P):
        o = out[k * _abi.ICP_OUT_STRIDE:(k + 1) * _abi.ICP_OUT_STRIDE]
        res.append(dict(T=o[0:16].astype(np.float32).reshape(4, 4), fitness=float(o[16]),
                        converged=bool(o[17]), iterations=int(o[18]),
                        state=_abi.ICP_STATES[int(o[19])], n_corr=int(o[20])))
    return res


def icp(fe: Frontend, src: torch.Tensor, tgt: torch.Tensor, params=None, guess=None):
    """One problem: icp.setInputSource(src); setInputTarget(tgt); align()."""
    hs = torch.tensor([0, int(src.shape[0])], dtype=torch.int64)
    ht = torch.tensor([0, int(tgt.shape[0])], dtype=torch.int64)
    return icp_batch(fe, src.contiguous(), hs.to(src.device), hs, tgt.contiguous(), ht.to(tgt.device),
                     ht, params, None if guess is None else [guess])[0]


def transform_cloud(xyzi: torch.Tensor, T) -> torch.Tensor:
    """pcl::transformPointCloud with an Affine3d: double arithmetic, float result, intensity
    kept."""
    Td = torch.as_tensor(np.asarray(T, np.float64), device=xyzi.device)
    p = xyzi[:, :3].double()
    out = xyzi.clone()
    out[:, :3] = (p @ Td[:3, :3].T + Td[:3, 3]).float()
    return out


# --------------------------------------------------------------------------- keyframe logic
@dataclass
class LoopConstraint:
    key_cur: int
    key_pre: int
    between: np.ndarray          # poseFrom.between(poseTo), 4x4
    noise: float                 # ICP fitness score (diagonal variances, :257-259)
    correction: np.ndarray       # correctionLidarFrame, 4x4


@dataclass
class LoopCloser:
    """The mapOptmization state machine for one sequence (keyframes, loop detection, ICP)."""
    fe: Frontend
    icp_leaf: float = 0.1
    radius: float = 15.0
    time_gap: float = 20.0
    search_num: int = 10
    key6d: list = field(default_factory=list)          # float32 [x, y, z, roll, pitch, yaw] + time
    key_frames: list = field(default_factory=list)     # device float4 plane clouds
    loop_index: dict = field(default_factory=dict)
    loop_record_index: int = 0
    trans_loop_adjust: np.ndarray = field(default_factory=lambda: np.eye(4))
    constraints: list = field(default_factory=list)

    def _T6(self, i):
        p = self.key6d[i]
        return get_transformation(*(float(v) for v in p[:6]))

    def is_key_frame(self, T_map_0_curr):
        """isKeyFrame (:129-144)."""
        if not self.key6d:
            return True
        tb = np.linalg.inv(self._T6(-1)) @ T_map_0_curr
        x, y, z, r, p, yw = get_translation_and_euler_angles(tb)
        return not (abs(r) < 0.01 and abs(p) < 0.01 and abs(yw) < 0.01 and math.sqrt(x * x + y * y + z * z) < 1)

    def detect_loop(self):
        """detectLoopFrameID (:167-197): radius search over key positions (nearest first)."""
        cur = len(self.key6d) - 1
        if cur in self.loop_index:
            return None
        pos = np.array([k[:3] for k in self.key6d], np.float32)
        d2 = ((pos - pos[cur]) ** 2).sum(1)
        cand = np.nonzero(d2 < np.float32(self.radius * self.radius))[0]   # FLANN: dist < r^2
        cand = cand[np.lexsort((cand, d2[cand]))]
        pre = -1
        for i in cand:
            if abs(self.key6d[i][6] - self.key6d[cur][6]) > self.time_gap:
                pre = int(i)
                break
        if pre == -1 or pre == cur:
            return None
        self.loop_record_index = cur + 2
        return cur, pre

    def local_map(self, key, n):
        """getLoopLocalMap (:200-218): keyframes key-n..key+n in the map frame, 0.1 m voxels."""
        parts = [transform_cloud(self.key_frames[k], self._T6(k))
                 for k in range(key - n, key + n + 1) if 0 <= k < len(self.key6d)]
        cloud = torch.cat(parts) if parts else torch.zeros(0, 4, device=self.fe.device)
        if cloud.shape[0] == 0:
            return cloud
        return voxel_grid_one(self.fe, cloud, self.icp_leaf)

    def add_loop_factor(self):
        """addLoopFactor (:221-272) up to the graph insertion."""
        n = len(self.key6d)
        if n < 5 or n - 1 <= self.loop_record_index:
            return None
        ids = self.detect_loop()
        if ids is None:
            return None
        cur, pre = ids
        cur_cloud = self.local_map(cur, 0)
        pre_cloud = self.local_map(pre, self.search_num)
        if cur_cloud.shape[0] < 300 or pre_cloud.shape[0] < 1000:
            return None
        r = icp(self.fe, cur_cloud, pre_cloud)
        if not r["converged"] or r["fitness"] > 0.2:
            return None
        corr = r["T"].astype(np.float64)
        self.loop_record_index += 30
        t_correct = corr @ self._T6(cur)
        pose_from = get_transformation(*get_translation_and_euler_angles(t_correct))
        c = LoopConstraint(cur, pre, between(pose_from, self._T6(pre)), float(np.float32(r["fitness"])), corr)
        self.loop_index[cur] = pre
        self.constraints.append(c)
        return c

    def process(self, plane_xyzi: torch.Tensor, q_xyzw, t, stamp: float):
        """One synchronised (/plane_frame_cloud2, /frame_odom2) pair (cloudThread :429-451 +
        mapOptimization :455-467).  Returns (T_map_0_curr, constraint or None, is_key)."""
        T = self.trans_loop_adjust @ pose_from_quat(q_xyzw, t)
        if not self.is_key_frame(T):
            return T, None, False
        x, y, z, r, p, yw = get_translation_and_euler_angles(T)
        self.key6d.append(np.array([x, y, z, r, p, yw], np.float32).tolist() + [float(stamp)])
        self.key_frames.append(plane_xyzi.contiguous())
        c = self.add_loop_factor()
        if c is not None:                                   # correctPoses (:321-326)
            self.trans_loop_adjust = self.trans_loop_adjust @ c.correction
        return T, c, True
