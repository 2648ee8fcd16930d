"""ssf -- MI355X (gfx950) SSF-SLAM LiDAR front-end.

Host-side mirror of the reference's hot-path interfaces over the C ABI in
include/ssf_frontend.h (libssf_frontend.so, hand-written HIP kernels).  There is no CPU
fallback anywhere in this package.
"""
from ._abi import SSFError  # noqa: F401
from .frontend import Frontend, PlaneBatch, frame_offsets, identity_poses  # noqa: F401
from .pose import mask_and_pose, slove_RT_by_SVD  # noqa: F401
from . import loop  # noqa: F401  (mapOptmization loop closure: voxel grid, ICP, LoopCloser)
from . import pointnet2  # noqa: F401  (TFlow point-set operators: pointutils surface)

__all__ = ["Frontend", "PlaneBatch", "frame_offsets", "identity_poses", "SSFError",
           "mask_and_pose", "slove_RT_by_SVD", "loop", "pointnet2"]
