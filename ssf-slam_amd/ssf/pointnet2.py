"""TFlow point-set operators on the GPU: the `lib.pointnet2_utils`
("pointutils") surface that scripts/ActiveSceneFlow/utils/utils.py:7 and utils/soflow.py:7
import, over the C ABI in include/ssf_pointnet2.h (hand-written HIP, csrc/pointnet2.hip).

Same names, argument order and layouts as the calls in the reference network:

    furthest_point_sample(xyz_t [B,N,3], npoint)            utils.py:226  -> int32 [B,npoint]
    gather_operation(features [B,C,N], idx [B,S])           utils.py:228  -> [B,C,S]
    knn(k, query [B,S,3], ref [B,N,3])                      utils.py:229  -> (dist, idx) [B,S,k]
    grouping_operation(features [B,C,N], idx [B,S,K])       utils.py:231  -> [B,C,S,K]
    three_nn(unknown [B,N,3], known [B,M,3])                utils.py:560  -> (dist, idx) [B,N,3]
    three_interpolate(features [B,C,M], idx, weight)        utils.py:662  -> [B,C,N]
    UpsampleFlow()(xyz [B,3,N], sparse_xyz [B,3,S], sparse_flow [B,C,S], k)  soflow.py:1442
    group_relative(xyz, new_xyz, points, idx)   utils.py:228-234 (grouping block, fused)

Inputs are CUDA tensors (float32 coordinates/features, integer indices); there is no CPU path.
Invalid arguments raise ValueError; a failing launch raises SSFError.
"""
from __future__ import annotations

import torch

from . import _abi
from .frontend import _ptr, _stream

__all__ = ["furthest_point_sample", "gather_operation", "knn", "grouping_operation", "three_nn",
           "three_interpolate", "upsample_flow", "UpsampleFlow", "group_relative"]


def _check(rc, what):
    if rc == 0:
        return
    msg = _abi.lib().ssf_pn2_last_error().decode(errors="replace")
    if rc == -1:
        raise ValueError(f"{what}: {msg}")
    raise _abi.SSFError(f"{what}: {msg}")


def _f32(t, name, dims):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA tensor")
    if t.dim() != dims:
        raise ValueError(f"{name} must have {dims} dimensions, got {tuple(t.shape)}")
    return t.detach().to(torch.float32).contiguous()


def _i32(t, name):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA tensor")
    return t.detach().to(torch.int32).contiguous()


def _bad_flag(device):
    return torch.zeros(1, dtype=torch.int32, device=device)


def _raise_if_bad(bad, check, what):
    if check and int(bad.item()) != 0:
        raise ValueError(f"{what}: index out of range")


def furthest_point_sample(xyz, npoint, start=None):
    """pointutils.furthest_point_sample (torch restatement: utils.py:68-89).  start: optional
    [B] first centroids (default 0)."""
    x = _f32(xyz, "xyz", 3)
    B, N, c3 = x.shape
    if c3 != 3:
        raise ValueError("xyz must be [B, N, 3]")
    out = torch.empty((B, int(npoint)), dtype=torch.int32, device=x.device)
    st = None
    if start is not None:
        st = _i32(torch.as_tensor(start, device=x.device), "start")
        if st.numel() != B:
            raise ValueError("start must hold one index per batch element")
    tmp = torch.empty((B, N), dtype=torch.float32, device=x.device) if N > 16384 else None
    rc = _abi.lib().ssf_pn2_furthest_point_sample(_stream(x.device), B, N, int(npoint), _ptr(x),
                                                  _ptr(st), _ptr(tmp), _ptr(out))
    _check(rc, "furthest_point_sample")
    return out


def knn(k, query, ref):
    """pointutils.knn(k, query, ref) (torch restatement knn_point, utils.py:92-108):
    -> (dist = sqrt of the squared distance, idx int32), both [B, S, k], ascending."""
    q = _f32(query, "query", 3)
    r = _f32(ref, "ref", 3)
    B, S, _ = q.shape
    if r.shape[0] != B or r.shape[2] != 3 or q.shape[2] != 3:
        raise ValueError("query [B, S, 3] and ref [B, N, 3] expected")
    N = r.shape[1]
    k = int(k)
    if not (0 < k <= _abi.PN2_KNN_MAX) or N == 0:
        raise ValueError(f"knn: need 0 < k <= {_abi.PN2_KNN_MAX} and a non-empty reference set")
    dist = torch.empty((B, S, k), dtype=torch.float32, device=q.device)
    idx = torch.empty((B, S, k), dtype=torch.int32, device=q.device)
    _check(_abi.lib().ssf_pn2_knn(_stream(q.device), B, S, N, k, _ptr(q), _ptr(r), _ptr(dist),
                                  _ptr(idx)), "knn")
    return dist, idx


def three_nn(unknown, known):
    """pointutils.three_nn(unknown [B,N,3], known [B,M,3]) -> (dist, idx) [B, N, 3]."""
    return knn(3, unknown, known)


def _gather(features, idx, check, what):
    f = _f32(features, "features", 3)
    ix = _i32(idx, "idx")
    B, Cc, N = f.shape
    if ix.shape[0] != B:
        raise ValueError(f"{what}: batch sizes differ")
    g = int(ix[0].numel()) if B else 0
    out = torch.empty((B, Cc) + tuple(ix.shape[1:]), dtype=torch.float32, device=f.device)
    bad = _bad_flag(f.device)
    _check(_abi.lib().ssf_pn2_gather(_stream(f.device), B, Cc, N, g, _ptr(f), _ptr(ix), _ptr(out),
                                     _ptr(bad)), what)
    _raise_if_bad(bad, check, what)
    return out


def gather_operation(features, idx, check=False):
    """pointutils.gather_operation(features [B,C,N], idx [B,S]) -> [B,C,S]."""
    return _gather(features, idx, check, "gather_operation")


def grouping_operation(features, idx, check=False):
    """pointutils.grouping_operation(features [B,C,N], idx [B,S,K]) -> [B,C,S,K]."""
    return _gather(features, idx, check, "grouping_operation")


def group_relative(xyz, new_xyz, points, idx, check=False):
    """The grouping block of PointNetSetAbstraction.forward (utils.py:228-234), one call:
    cat([grouping_operation(xyz, idx) - new_xyz.unsqueeze(-1), grouping_operation(points, idx)],
    dim=1).  xyz [B,3,N] (N <= 36864), new_xyz [B,3,S], points [B,C,N] or None, idx [B,S,K]
    -> [B, 3 + C, S, K]."""
    x = _f32(xyz, "xyz", 3)
    nx = _f32(new_xyz, "new_xyz", 3)
    ix = _i32(idx, "idx")
    B, c3, N = x.shape
    if c3 != 3 or nx.shape[:2] != (B, 3) or ix.dim() != 3 or ix.shape[:2] != (B, nx.shape[2]):
        raise ValueError("xyz [B,3,N], new_xyz [B,3,S] and idx [B,S,K] expected")
    S, K = ix.shape[1], ix.shape[2]
    f = None
    Cc = 0
    if points is not None:
        f = _f32(points, "points", 3)
        if f.shape[0] != B or f.shape[2] != N:
            raise ValueError("points must be [B, C, N]")
        Cc = f.shape[1]
    out = torch.empty((B, 3 + Cc, S, K), dtype=torch.float32, device=x.device)
    bad = _bad_flag(x.device)
    _check(_abi.lib().ssf_pn2_group_relative(_stream(x.device), B, N, S, K, Cc, _ptr(x), _ptr(nx),
                                             _ptr(f), _ptr(ix), _ptr(out), _ptr(bad)),
           "group_relative")
    _raise_if_bad(bad, check, "group_relative")
    return out


def three_interpolate(features, idx, weight, check=False):
    """pointutils.three_interpolate(features [B,C,M], idx [B,N,3], weight [B,N,3]) -> [B,C,N]."""
    f = _f32(features, "features", 3)
    ix = _i32(idx, "idx")
    w = _f32(weight, "weight", 3)
    B, Cc, M = f.shape
    if ix.shape != w.shape or ix.dim() != 3 or ix.shape[0] != B or ix.shape[2] != 3:
        raise ValueError("idx and weight must both be [B, N, 3]")
    N = ix.shape[1]
    out = torch.empty((B, Cc, N), dtype=torch.float32, device=f.device)
    bad = _bad_flag(f.device)
    _check(_abi.lib().ssf_pn2_three_interpolate(_stream(f.device), B, Cc, M, N, _ptr(f), _ptr(ix),
                                                _ptr(w), _ptr(out), _ptr(bad)), "three_interpolate")
    _raise_if_bad(bad, check, "three_interpolate")
    return out


def upsample_flow(xyz, sparse_xyz, sparse_flow, k=3):
    """UpsampleFlow.forward (soflow.py:1442-1470), one fused kernel: xyz [B,3,N],
    sparse_xyz [B,3,S] (S <= 4096), sparse_flow [B,C,S] -> [B,C,N]."""
    x = _f32(xyz, "xyz", 3)
    sx = _f32(sparse_xyz, "sparse_xyz", 3)
    sf = _f32(sparse_flow, "sparse_flow", 3)
    B, c3, N = x.shape
    S = sx.shape[2]
    if c3 != 3 or sx.shape[:2] != (B, 3) or sf.shape[0] != B or sf.shape[2] != S:
        raise ValueError("xyz [B,3,N], sparse_xyz [B,3,S], sparse_flow [B,C,S] expected")
    if not (0 < S <= _abi.PN2_UPSAMPLE_MAX_SPARSE) or not (0 < int(k) <= 16):
        raise ValueError(f"upsample_flow: need 0 < S <= {_abi.PN2_UPSAMPLE_MAX_SPARSE}, 0 < k <= 16")
    out = torch.empty((B, sf.shape[1], N), dtype=torch.float32, device=x.device)
    _check(_abi.lib().ssf_pn2_upsample_flow(_stream(x.device), B, N, S, sf.shape[1], int(k),
                                            _ptr(x), _ptr(sx), _ptr(sf), _ptr(out)),
           "upsample_flow")
    return out


class UpsampleFlow(torch.nn.Module):
    """soflow.py:1442 UpsampleFlow (no parameters): forward(xyz, sparse_xyz, sparse_flow, k=3)."""

    def forward(self, xyz, sparse_xyz, sparse_flow, k=3):
        return upsample_flow(xyz, sparse_xyz, sparse_flow, k)
