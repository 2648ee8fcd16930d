"""Golden vectors for the TFlow point-set operators, produced by the
REFERENCE's own torch restatements of the un-vendored `lib.pointnet2_utils` extension.

Run in the build container only (it reads /root/reference, absent on the GPU box); the .npz it
writes is committed and is what tests/test_oracle_pn2.py and tests/test_gpu_pointnet2.py read.

What is imported / called:
  * /root/reference/scripts/ActiveSceneFlow/utils/utils.py, with `lib` / `lib.pointnet2_utils`
    (imported at module level, :7, never called by the functions used here) replaced by empty
    stubs.  Called: farthest_point_sample (:68-89, torch RNG seeded), knn_point (:92-108),
    index_points (:48-65).
  * utils/soflow.py is NOT importable (torch_scatter is absent), so UpsampleFlow.forward
    (:1442-1470) is composed here from the imported knn_point / index_points, line by line,
    and the weighted 3-NN sum of PointNetFeaturePropogation (utils.py:658-663) likewise.

Inputs: two seeded synthetic 64-beam scans (ssf.synth), subsampled to 2048 points.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_UTILS = "/root/reference/scripts/ActiveSceneFlow/utils/utils.py"
sys.path.insert(0, os.path.join(REPO, "ssf-slam_amd"))


def import_reference():
    lib = types.ModuleType("lib")
    lib.pointnet2_utils = types.ModuleType("lib.pointnet2_utils")
    sys.modules.setdefault("lib", lib)
    sys.modules.setdefault("lib.pointnet2_utils", lib.pointnet2_utils)
    spec = importlib.util.spec_from_file_location("ref_asf_utils", REF_UTILS)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    import torch
    from ssf import synth

    U = import_reference()
    rng = np.random.default_rng(20240417)
    B, N, NPOINT, K = 2, 2048, 256, 16
    clouds = []
    for b in range(B):
        f = synth.scan(7, b, n_az=300)
        p = f["pos1"].numpy().astype(np.float32)
        sel = np.sort(rng.choice(p.shape[0], N, replace=False))
        clouds.append(p[sel])
    xyz = np.stack(clouds)                                          # [B, N, 3]
    xt = torch.from_numpy(xyz)

    torch.manual_seed(1234)
    fps = U.farthest_point_sample(xt, NPOINT)                        # [B, NPOINT] long
    new_xyz = U.index_points(xt, fps)                                # [B, NPOINT, 3]
    kd, ki = U.knn_point(K, xt, new_xyz)                             # [B, NPOINT, K]
    feat = rng.standard_normal((B, 8, N)).astype(np.float32)         # [B, C, N]
    ft = torch.from_numpy(feat)
    gathered = U.index_points(ft.permute(0, 2, 1), fps).permute(0, 2, 1)        # gather_operation
    grouped = U.index_points(ft.permute(0, 2, 1), ki).permute(0, 3, 1, 2)       # grouping_operation

    # weighted 3-NN sum (utils.py:658-663): dense = all N points, known = the NPOINT centroids
    d3, i3 = U.knn_point(3, new_xyz, xt)                             # three_nn(pos1_t, pos2_t)
    d3c = d3.clone()
    d3c[d3c < 1e-10] = 1e-10
    w3 = 1.0 / d3c
    w3 = w3 / torch.sum(w3, -1, keepdim=True)
    sfeat = torch.from_numpy(rng.standard_normal((B, 4, NPOINT)).astype(np.float32))
    g3 = U.index_points(sfeat.permute(0, 2, 1), i3).permute(0, 3, 1, 2)        # [B, C, N, 3]
    interp = torch.sum(g3 * w3.view(B, 1, N, 3), dim=-1)

    # UpsampleFlow.forward (soflow.py:1442-1470), k = 3 and k = 5
    xyz_c = xt.permute(0, 2, 1).contiguous()                        # [B, 3, N]
    sxyz_c = new_xyz.permute(0, 2, 1).contiguous()                  # [B, 3, S]
    sflow = torch.from_numpy((rng.standard_normal((B, 3, NPOINT)) * 0.5).astype(np.float32))
    ups = {}
    for k in (3, 5):
        _, knn_idx = U.knn_point(k, new_xyz, xt)                     # :1458-1461
        grouped_xyz_norm = U.index_points(sxyz_c.permute(0, 2, 1), knn_idx).permute(0, 3, 1, 2) \
            - xyz_c.view(B, 3, N, 1)                                 # :1462
        dist = torch.norm(grouped_xyz_norm, dim=1).clamp(min=1e-10)  # :1463
        norm = torch.sum(1.0 / dist, dim=-1, keepdim=True)           # :1464
        weight = (1.0 / dist) / norm                                 # :1465
        grouped_flow = U.index_points(sflow.permute(0, 2, 1), knn_idx).permute(0, 3, 1, 2)
        dense = torch.sum(weight.view(B, 1, N, k) * grouped_flow, dim=-1)
        ups[k] = (knn_idx.numpy().astype(np.int32), dense.clamp(-100.0, 100.0).numpy())

    out = os.path.join(HERE, "pn2_ref.npz")
    np.savez_compressed(
        out, xyz=xyz, fps_start=fps[:, 0].numpy().astype(np.int32),
        fps_idx=fps.numpy().astype(np.int32), knn_k=np.int32(K), knn_dist=kd.numpy(),
        knn_idx=ki.numpy().astype(np.int32), feat=feat, gathered=gathered.numpy(),
        grouped=grouped.numpy(), three_dist=d3.numpy(), three_idx=i3.numpy().astype(np.int32),
        three_weight=w3.numpy(), sfeat=sfeat.numpy(), interp=interp.numpy(),
        sflow=sflow.numpy(), up3_idx=ups[3][0], up3=ups[3][1], up5_idx=ups[5][0], up5=ups[5][1])
    print("wrote", out)


if __name__ == "__main__":
    main()
