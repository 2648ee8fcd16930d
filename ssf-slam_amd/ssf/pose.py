"""Reference-named Python entry points of the SSF pose block, GPU-backed.

scripts/PointCloudOdometry_noSeg.py (and PointCloudOdometry.py, main_sju_occ_ros.py:256-284)
computes, per frame:

    X = concatenate((move_gt, points), axis=1)                 # :97
    all_label = GaussianMixture(n_components=2).fit_predict(X) # :98-101
    bg_label = Counter(all_label).most_common(1)[0][0]         # :102
    R, t = slove_RT_by_SVD(points[bg] + move_gt[bg], points[bg])   # :114-118
    q = Quaternion(matrix=R); publish [t, q.x, q.y, q.z, q.w]  # :119-125

`mask_and_pose` runs that whole block in one HIP kernel (k_mask_pose) for one or many frames;
`slove_RT_by_SVD` keeps the reference signature.  Error behaviour: the reference raises
TypeError when det(R) < 0 (`Vt.T & U.T`, :33) and pyquaternion raises ValueError for a
non-orthogonal R; here both raise ValueError (reflection='fix' applies the evident intent of
:32-33 instead).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _abi
from .frontend import Frontend, frame_offsets

_FE: dict = {}


def _frontend(device) -> Frontend:
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else
                       (device.index if isinstance(device, torch.device) else int(device)))
    fe = _FE.get(dev.index)
    if fe is None:
        fe = _FE[dev.index] = Frontend(64, device=dev.index)
    return fe


def _is_f64(a) -> bool:
    return (a.dtype == torch.float64) if isinstance(a, torch.Tensor) else (np.asarray(a).dtype == np.float64)


def _as_dev(a, dev, dtype):
    if isinstance(a, torch.Tensor):
        return a.to(dev, dtype).contiguous()
    npd = np.float64 if dtype == torch.float64 else np.float32
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a), dtype=npd)).to(dev)


def _storage(*arrays):
    """float64 when any input is float64 (the reference then computes in f64 throughout; the
    f64 kernel loads those values exactly), else float32 (LiDAR data)."""
    return torch.float64 if any(_is_f64(a) for a in arrays) else torch.float32


def _raise_status(st):
    st = int(st)
    if st == _abi.POSE_REFLECTION:
        raise ValueError("slove_RT_by_SVD: reflection (det(R) < 0); the reference raises TypeError here")
    if st == _abi.POSE_NOT_ORTHOGONAL:
        raise ValueError("Matrix must be orthogonal, i.e. its transpose should be its inverse")
    if st == _abi.POSE_EMPTY:
        raise ValueError("no background points")
    if st == _abi.POSE_SYNC_FAILED:
        raise RuntimeError("mask kernel: a frame part never arrived at an exchange (sync timeout)")
    if st == _abi.POSE_GMM_FAILED:
        raise ValueError("Fitting the mixture model failed (ill-defined empirical covariance)")


def _check_kabsch_dtype(kabsch_dtype):
    if kabsch_dtype not in ("float64", "float32"):
        raise ValueError(f"kabsch_dtype must be 'float64' or 'float32', not {kabsch_dtype!r}")


def slove_RT_by_SVD(src, dst, reflection: str = "raise", device=None, kabsch_dtype: str = "float64"):
    """R (3,3), t (3,1) minimising |R src + t - dst| (reference signature, float64 results).
    float64 inputs run the f64-storage kernel (no input rounding); float32 inputs the f32 one.
    The kernel takes (pos, flow) = (dst, src - dst) and forms src = pos + flow in f64: exact
    for f32 inputs, and within an ulp of src for f64 inputs.
    kabsch_dtype "float32": numpy's float32 arithmetic on float32 arrays (ssf_kabsch_f32_batch;
    the inputs are rounded to float32 first), R / t hold float32 values."""
    _check_kabsch_dtype(kabsch_dtype)
    fe = _frontend(device)
    if kabsch_dtype == "float32":
        dst_t = _as_dev(dst, fe.device, torch.float32)
        src_t = _as_dev(src, fe.device, torch.float32)
        off, h_off = frame_offsets([dst_t.shape[0]], fe.device)
        o = fe.kabsch_f32(dst_t, off, h_off, src=src_t, reflection=1 if reflection == "fix" else 0)[0].cpu().numpy()
        if int(o[_abi.POSE_OUT["STATUS"]]) == _abi.POSE_REFLECTION and reflection != "fix":
            _raise_status(o[_abi.POSE_OUT["STATUS"]])
        return o[7:16].reshape(3, 3).copy(), o[0:3].reshape(3, 1).copy()
    dt = _storage(src, dst)
    dst_t = _as_dev(dst, fe.device, dt)
    src_t = _as_dev(src, fe.device, dt)
    flow = (src_t - dst_t).contiguous()
    off, h_off = frame_offsets([dst_t.shape[0]], fe.device)
    ones = torch.ones(dst_t.shape[0], dtype=torch.uint8, device=fe.device)
    out, _ = fe.mask_pose(dst_t, flow, off, h_off, mode="given", mask_in=ones,
                          reflection=1 if reflection == "fix" else 0, want_mask=False)
    o = out[0].cpu().numpy()
    if int(o[_abi.POSE_OUT["STATUS"]]) == _abi.POSE_REFLECTION and reflection != "fix":
        _raise_status(o[_abi.POSE_OUT["STATUS"]])
    R = o[7:16].reshape(3, 3).copy()
    t = o[0:3].reshape(3, 1).copy()
    return R, t


class MaskPose(tuple):
    """(R, t, q_xyzw, bg_mask): the Python boundary of SURVEY §8(b).  One frame: R (3, 3) and
    t (3, 1) as slove_RT_by_SVD returns them, q_xyzw (4,), bg_mask (device uint8); F frames (with
    frame_sizes): the same with a leading F axis.  The batched fields are also readable by key
    or attribute -- res["R"] [F, 3, 3], res["t"] [F, 3], res["q_xyzw"] [F, 4], res["para_t_q"]
    [F, 7] (the published [t, q]), res["bg_mask"], res["info"] (iteration counts, labels,
    k-means++ centres, lower bound)."""
    def __new__(cls, values, fields):
        obj = super().__new__(cls, values)
        obj._fields = fields
        return obj

    def __getitem__(self, k):
        return self._fields[k] if isinstance(k, str) else super().__getitem__(k)

    def __getattr__(self, k):
        if k.startswith("_"):
            raise AttributeError(k)
        try:
            return self._fields[k]
        except KeyError:
            raise AttributeError(k) from None

    def keys(self):
        return self._fields.keys()


def mask_and_pose(points, flow, mode: str = "gmm", gt_mask=None, seed: int | None = None,
                  draws=None, reflection: str = "raise", device=None, frame_sizes=None,
                  kabsch_dtype: str = "float64", errors: str = "raise"):
    """The PointCloudOdometry_noSeg.py:97-125 block for one frame (or F frames packed back to
    back with `frame_sizes`).  mode 'gmm' (GaussianMixture on [flow, xyz]), 'gt'
    (background = s_fg_mask == 0, PointCloudOdometry.py:91) or 'given' (background = mask != 0).
    kabsch_dtype "float64" (default): the Kabsch + quaternion tail in f64, the reference's
    arithmetic on float64 arrays; "float32": the reference's float32 arithmetic, as the ASF block
    runs it on float32 network flow (main_sju_occ_ros.py:273-284; inputs stored as float32,
    ssf_kabsch_f32_batch after the mask kernel, same stream).
    errors "raise" (default): a frame whose pose fails raises as the reference does (one frame,
    one call); "status": nothing raises, info["status"] holds every frame's status (0 or a
    POSE_* code) -- a batch keeps its good frames when one frame fails, e.g. a float32 R whose
    orthogonality test (atol 1e-8) sits at the rounding level.
    -> MaskPose: (R, t, q_xyzw, bg_mask), plus keyed batched fields (see MaskPose)."""
    _check_kabsch_dtype(kabsch_dtype)
    if errors not in ("raise", "status"):
        raise ValueError(f"errors must be 'raise' or 'status', not {errors!r}")
    fe = _frontend(device)
    dt = torch.float32 if kabsch_dtype == "float32" else _storage(points, flow)
    pts = _as_dev(points, fe.device, dt)
    fl = _as_dev(flow, fe.device, dt)
    sizes = [pts.shape[0]] if frame_sizes is None else list(frame_sizes)
    off, h_off = frame_offsets(sizes, fe.device)
    if seed is not None:
        fe.seed(seed)
    m = None
    if mode != "gmm":
        if gt_mask is None:
            raise ValueError(f"mode {mode!r} needs gt_mask")
        m = torch.as_tensor(np.asarray(gt_mask) if not isinstance(gt_mask, torch.Tensor) else gt_mask)
        m = m.to(fe.device, torch.uint8).contiguous()
    out, bg = fe.mask_pose(pts, fl, off, h_off, mode=mode, mask_in=m, draws=draws,
                           reflection=1 if reflection == "fix" else 0)
    if kabsch_dtype == "float32":
        fe.kabsch_f32(pts, off, h_off, flow=fl, mask=bg, reflection=1 if reflection == "fix" else 0,
                      out=out)
    o = out.cpu().numpy()
    status = o[:, _abi.POSE_OUT["STATUS"]].astype(np.int32)
    if errors == "raise":
        for st in status:
            if int(st) != 0:
                _raise_status(st)
    fields = dict(R=o[:, 7:16].reshape(-1, 3, 3), t=o[:, 0:3], q_xyzw=o[:, 3:7],
                  para_t_q=o[:, 0:7], bg_mask=bg,
                  info=dict(bg_label=o[:, 18], n_bg=o[:, 17], kmeans_iter=o[:, 19], em_iter=o[:, 20],
                            converged=o[:, 21], centers=o[:, 22:24], lower_bound=o[:, 24],
                            passes=o[:, 25], status=status))
    R, t, q = fields["R"].copy(), fields["t"].reshape(-1, 3, 1).copy(), fields["q_xyzw"].copy()
    if frame_sizes is None:                      # one frame: the shapes of slove_RT_by_SVD
        R, t, q = R[0], t[0], q[0]
    return MaskPose((R, t, q, bg), fields)
