"""TFlow point-set operators on the GPU (csrc/pointnet2.hip through
include/ssf_pointnet2.h) vs the golden vectors from the reference's own torch operators
(tests/golden/pn2_ref.npz) and vs the CPU oracle (oracle/pn2_oracle.c) on larger TFlow shapes.

Bars: furthest point sampling, k-NN / three_nn indices, gather / grouping and
three_interpolate are bit-exact against the oracle (same f32 expressions, no FMA, IEEE sqrt and
division); k-NN distances are within 1 ulp of the golden vectors (torch's CPU sqrt is not
correctly rounded, see tests/test_oracle_pn2.py); UpsampleFlow within rtol 1e-5 of the golden
vectors (torch.norm / torch.sum reduction order) and bit-exact against the oracle.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "pn2_ref.npz")


@pytest.fixture(scope="module")
def g():
    return dict(np.load(GOLD))


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def test_golden_fps_knn_gather(g, dev):
    from ssf import pointnet2 as P
    xyz = _t(g["xyz"], dev)
    fps = P.furthest_point_sample(xyz, g["fps_idx"].shape[1], start=_t(g["fps_start"], dev))
    assert np.array_equal(fps.cpu().numpy(), g["fps_idx"])
    new_xyz = torch.gather(xyz, 1, fps.long().unsqueeze(-1).expand(-1, -1, 3)).contiguous()
    d, i = P.knn(int(g["knn_k"]), new_xyz, xyz)
    assert np.array_equal(i.cpu().numpy(), g["knn_idx"])
    np.testing.assert_allclose(d.cpu().numpy(), g["knn_dist"], rtol=2.5e-7, atol=0)
    d3, i3 = P.three_nn(xyz, new_xyz)
    assert np.array_equal(i3.cpu().numpy(), g["three_idx"])
    np.testing.assert_allclose(d3.cpu().numpy(), g["three_dist"], rtol=2.5e-7, atol=0)
    feat = _t(g["feat"], dev)
    assert np.array_equal(P.gather_operation(feat, fps, check=True).cpu().numpy(), g["gathered"])
    assert np.array_equal(P.grouping_operation(feat, i, check=True).cpu().numpy(), g["grouped"])
    interp = P.three_interpolate(_t(g["sfeat"], dev), _t(g["three_idx"], dev),
                                 _t(g["three_weight"], dev), check=True)
    np.testing.assert_allclose(interp.cpu().numpy(), g["interp"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("k", [3, 5])
def test_golden_upsample_flow(g, dev, oracle, k):
    from ssf import pointnet2 as P
    xyz = np.ascontiguousarray(g["xyz"].transpose(0, 2, 1))
    new_xyz = np.take_along_axis(g["xyz"], g["fps_idx"][..., None].astype(np.int64), axis=1)
    sxyz = np.ascontiguousarray(new_xyz.transpose(0, 2, 1))
    got = P.UpsampleFlow()(_t(xyz, dev), _t(sxyz, dev), _t(g["sflow"], dev), k=k).cpu().numpy()
    np.testing.assert_allclose(got, g[f"up{k}"], rtol=1e-5, atol=1e-6)
    assert np.array_equal(got, oracle.pn2_upsample_flow(xyz, sxyz, g["sflow"], k=k))


def _cloud(rng, b, n, scale=20.0):
    x = rng.standard_normal((b, n, 3)).astype(np.float32) * np.float32(scale)
    return x


@pytest.mark.parametrize("n,npoint", [(8192, 2048), (2048, 512), (700, 700), (12000, 1000), (20000, 256), (5, 1)])
def test_fps_vs_oracle(dev, oracle, n, npoint):
    from ssf import pointnet2 as P
    rng = np.random.default_rng(n)
    x = _cloud(rng, 2, n)
    start = np.array([0, n // 3], np.int32)
    got = P.furthest_point_sample(_t(x, dev), npoint, start=_t(start, dev)).cpu().numpy()
    assert np.array_equal(got, oracle.pn2_fps(x, npoint, start=start))


def test_fps_duplicates_and_ties(dev, oracle):
    """exact duplicates and equal distances: the lowest index wins, as torch.max"""
    from ssf import pointnet2 as P
    g = np.stack(np.meshgrid(np.arange(8), np.arange(8), np.arange(4), indexing="ij"), -1)
    x = np.repeat(g.reshape(1, -1, 3).astype(np.float32), 2, axis=1)    # every point twice
    got = P.furthest_point_sample(_t(x, dev), 200).cpu().numpy()
    assert np.array_equal(got, oracle.pn2_fps(x, 200))


@pytest.mark.parametrize("k,s,n", [(16, 2048, 8192), (1, 300, 5000), (8, 512, 2048),
                                   (20, 100, 3000), (32, 64, 4500), (16, 10, 7)])
def test_knn_vs_oracle(dev, oracle, k, s, n):
    from ssf import pointnet2 as P
    rng = np.random.default_rng(k * 1000 + s)
    ref = _cloud(rng, 2, n)
    q = _cloud(rng, 2, s)
    q[:, : min(s, n) // 2] = ref[:, : min(s, n) // 2]        # queries on reference points (d = 0)
    d, i = P.knn(k, _t(q, dev), _t(ref, dev))
    od, oi = oracle.pn2_knn(k, q, ref)
    assert np.array_equal(i.cpu().numpy(), oi)
    assert np.array_equal(d.cpu().numpy(), od)


def test_knn_ties_lower_index_first(dev, oracle):
    from ssf import pointnet2 as P
    ref = np.repeat(np.arange(40, dtype=np.float32).reshape(1, -1, 1), 3, axis=2)
    ref = np.concatenate([ref, ref], axis=1)                   # duplicates at i and i + 40
    q = ref[:, ::7].copy()
    d, i = P.knn(6, _t(q, dev), _t(ref, dev))
    od, oi = oracle.pn2_knn(6, q, ref)
    assert np.array_equal(i.cpu().numpy(), oi) and np.array_equal(d.cpu().numpy(), od)
    assert (oi[0, :, 0] < 40).all() and (oi[0, :, 1] == oi[0, :, 0] + 40).all()


def test_group_interp_vs_oracle(dev, oracle):
    from ssf import pointnet2 as P
    rng = np.random.default_rng(5)
    B, C, N, S, K = 2, 64, 8192, 2048, 16
    feat = rng.standard_normal((B, C, N)).astype(np.float32)
    idx = rng.integers(0, N, (B, S, K)).astype(np.int32)
    out = P.grouping_operation(_t(feat, dev), _t(idx, dev), check=True).cpu().numpy()
    assert np.array_equal(out, oracle.pn2_gather(feat, idx))
    i3 = rng.integers(0, S, (B, N, 3)).astype(np.int32)
    w3 = rng.uniform(0, 1, (B, N, 3)).astype(np.float32)
    sf = rng.standard_normal((B, C, S)).astype(np.float32)
    got = P.three_interpolate(_t(sf, dev), _t(i3, dev), _t(w3, dev), check=True).cpu().numpy()
    assert np.array_equal(got, oracle.pn2_three_interpolate(sf, i3, w3))
    bad = idx.copy()
    bad[1, 3, 2] = N
    with pytest.raises(ValueError):
        P.grouping_operation(_t(feat, dev), _t(bad, dev), check=True)


@pytest.mark.parametrize("k,s,n,c", [(7, 2048, 8192, 3), (3, 128, 256, 64), (5, 4096, 1000, 1),
                                     (16, 10, 50, 2)])
def test_upsample_vs_oracle(dev, oracle, k, s, n, c):
    from ssf import pointnet2 as P
    rng = np.random.default_rng(k + s)
    xyz = _cloud(rng, 2, n).transpose(0, 2, 1).copy()
    sxyz = _cloud(rng, 2, s).transpose(0, 2, 1).copy()
    sxyz[:, :, :5] = xyz[:, :, :5]                             # coincident points: 1e-10 clamp
    sf = (rng.standard_normal((2, c, s)) * 60).astype(np.float32)   # some sums hit the +-100 clamp
    got = P.upsample_flow(_t(xyz, dev), _t(sxyz, dev), _t(sf, dev), k=k).cpu().numpy()
    assert np.array_equal(got, oracle.pn2_upsample_flow(xyz, sxyz, sf, k=k))


@pytest.mark.parametrize("c,n,s,k", [(35, 8192, 2048, 16), (3, 40000, 512, 8), (130, 300, 77, 5)])
def test_group_staging_paths_vs_oracle(dev, oracle, c, n, s, k):
    """LDS-staged rows (channel groups not dividing C) and the global fallback (n > 36864)"""
    from ssf import pointnet2 as P
    rng = np.random.default_rng(c + n)
    feat = rng.standard_normal((2, c, n)).astype(np.float32)
    idx = rng.integers(0, n, (2, s, k)).astype(np.int32)
    out = P.grouping_operation(_t(feat, dev), _t(idx, dev), check=True).cpu().numpy()
    assert np.array_equal(out, oracle.pn2_gather(feat, idx))
    g1 = P.gather_operation(_t(feat, dev), _t(idx[:, :, 0], dev), check=True).cpu().numpy()
    assert np.array_equal(g1, oracle.pn2_gather(feat, np.ascontiguousarray(idx[:, :, 0])))
    i3 = rng.integers(0, n, (2, s, 3)).astype(np.int32)
    w3 = rng.uniform(0, 1, (2, s, 3)).astype(np.float32)
    got = P.three_interpolate(_t(feat, dev), _t(i3, dev), _t(w3, dev), check=True).cpu().numpy()
    assert np.array_equal(got, oracle.pn2_three_interpolate(feat, i3, w3))
    i3[0, 1, 1] = -1
    with pytest.raises(ValueError):
        P.three_interpolate(_t(feat, dev), _t(i3, dev), _t(w3, dev), check=True)


@pytest.mark.parametrize("c,n,s,k", [(32, 8192, 2048, 16), (0, 2048, 512, 16), (128, 512, 256, 8)])
def test_group_relative_vs_oracle(dev, oracle, c, n, s, k):
    """PointNetSetAbstraction grouping block (utils.py:228-234): cat(grouped xyz - centroid,
    grouped features), bit-exact vs the oracle gathers + one f32 subtraction"""
    from ssf import pointnet2 as P
    rng = np.random.default_rng(c + s)
    xyz = _cloud(rng, 2, n).transpose(0, 2, 1).copy()                    # [B, 3, N]
    fps = oracle.pn2_fps(np.ascontiguousarray(xyz.transpose(0, 2, 1)), s)
    new_xyz = oracle.pn2_gather(xyz, fps)                                # [B, 3, S]
    _, idx = oracle.pn2_knn(k, np.ascontiguousarray(new_xyz.transpose(0, 2, 1)),
                            np.ascontiguousarray(xyz.transpose(0, 2, 1)))
    feat = rng.standard_normal((2, c, n)).astype(np.float32) if c else None
    got = P.group_relative(_t(xyz, dev), _t(new_xyz, dev), None if feat is None else _t(feat, dev),
                           _t(idx, dev), check=True).cpu().numpy()
    want = oracle.pn2_gather(xyz, idx) - new_xyz[..., None]
    if c:
        want = np.concatenate([want, oracle.pn2_gather(feat, idx)], axis=1)
    assert got.shape == (2, 3 + c, s, k)
    assert np.array_equal(got, want)


def test_large_batch_launch_paths_vs_oracle(dev, oracle):
    """b * ceil(s / 256) >= 512: the 256-thread k-NN / UpsampleFlow launches (the small-batch
    64-thread ones are covered above)"""
    from ssf import pointnet2 as P
    rng = np.random.default_rng(64)
    ref = _cloud(rng, 64, 512)
    q = _cloud(rng, 64, 2048)
    d, i = P.knn(16, _t(q, dev), _t(ref, dev))
    od, oi = oracle.pn2_knn(16, q, ref)
    assert np.array_equal(i.cpu().numpy(), oi) and np.array_equal(d.cpu().numpy(), od)
    xyz = _cloud(rng, 64, 2048).transpose(0, 2, 1).copy()
    sxyz = _cloud(rng, 64, 128).transpose(0, 2, 1).copy()
    sf = rng.standard_normal((64, 2, 128)).astype(np.float32)
    got = P.upsample_flow(_t(xyz, dev), _t(sxyz, dev), _t(sf, dev), k=3).cpu().numpy()
    assert np.array_equal(got, oracle.pn2_upsample_flow(xyz, sxyz, sf, k=3))
