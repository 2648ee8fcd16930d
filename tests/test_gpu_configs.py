"""BASELINE.json configs at their own sizes, through the C ABI, against the oracle.

configs[2] -- PointCloudOdometry_noSeg.py path with the scene-flow mask applied before the
features: 32 consecutive 120k-point pairs of one synthetic sequence.  The GMM mask + Kabsch of all
33 frames run in ONE launch (seeded RandomState draws, PointCloudOdometry_noSeg.py:97-125), the
background points feed frameFeature (beyond the reference, whose frameFeature sees every point,
:92-94; parity = the reference extraction of the compacted cloud), then the 32 pairs are registered
in order with the warm start chained (lidarOdometry_onlyPC.cpp:164, 251-252) and accumulated.

configs[4] -- 256k-point scans (64 beams x 4000 azimuth steps): features bit-exact, plane table
bit-exact, the association above the LDS staging size index-exact, GN poses, and mask + Kabsch.

Bars as everywhere: float stages bit-exact, poses <= 1e-5 m / 1e-6 rad per pair, mask labels
>= 99.9 % (identical in practice), Kabsch t <= 1e-5 m.
"""
import numpy as np
import pytest
import torch

from helpers import frame

pytestmark = pytest.mark.gpu

TOL_T, TOL_R = 1e-5, 1e-6


def _angle(q1, q2):
    d = abs(float(np.dot(q1 / np.linalg.norm(q1), q2 / np.linalg.norm(q2))))
    return 2.0 * np.arccos(min(1.0, d))


def _pair(pb, a, b):
    import ssf
    last = ssf.PlaneBatch(pb.xyzi, pb.count[a:a + 1], pb.off[a:a + 2], pb.h_off[a:a + 2], pb.max_points)
    curr = ssf.PlaneBatch(pb.xyzi, pb.count[b:b + 1], pb.off[b:b + 2], pb.h_off[b:b + 2], pb.max_points)
    return last, curr


def test_config2_noseg_mask_before_features_32_pairs(oracle, dev):
    import ssf
    F = 33
    frames = [frame(8, k, n_az=1875) for k in range(F)]
    N = frames[0][0].shape[0]
    pos = torch.from_numpy(np.concatenate([f[0] for f in frames])).to(dev)
    flow = torch.from_numpy(np.concatenate([f[1] for f in frames])).to(dev)
    off, h_off = ssf.frame_offsets([N] * F, dev)
    rs = oracle.LegacyRandomState(20240000)
    draws = np.stack([rs.random_sample(3) for _ in range(F)])
    fe = ssf.Frontend(64, device=dev.index or 0, solver="gn", max_iter=10)
    out, bg = fe.mask_pose(pos, flow, off, h_off, mode="gmm", draws=draws)
    pb = fe.extract_planes_batch(pos, off, h_off, keep=bg)
    table = fe.plane_table(pb)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    bgh = bg.cpu().numpy()
    # mask + Kabsch of every frame vs the oracle (same draws)
    for k in range(F):
        ref = oracle.mask_and_pose(frames[k][0], frames[k][1], draws[k])
        assert ref["rc"] == 0 and int(o[k, 16]) == 0, k
        agree = (bgh[k * N:(k + 1) * N] == ref["bg_mask"]).mean()
        assert agree >= 0.999, (k, agree)
        assert np.abs(o[k, 0:3] - ref["t"]).max() < TOL_T, k
        assert _angle(o[k, 3:7], ref["q_xyzw"]) < TOL_R, k
    # masked features: the reference extraction of the compacted background cloud, bit for bit
    planes = []
    for k in range(F):
        keep = bgh[k * N:(k + 1) * N] != 0
        ref = oracle.extract_planes(frames[k][0][keep], 64)
        got = pb.frame(k).cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), k
        planes.append(ref)
    # 32 consecutive pairs, warm start chained, accumulated on the device
    rel = ssf.identity_poses(1, dev)
    ab = ssf.identity_poses(1, dev)
    q_abs, t_abs = np.array([0.0, 0, 0, 1]), np.zeros(3)
    for k in range(1, F):
        q0 = rel[0, :4].cpu().numpy().copy()
        t0 = rel[0, 4:].cpu().numpy().copy()
        last, curr = _pair(pb, k - 1, k)
        res = fe.register(last, table, curr, rel, ab, want_log=True)
        torch.cuda.synchronize()
        q, t, log, c = oracle.register_pair(planes[k - 1], planes[k], 0.05, mode=oracle.MODE_GN,
                                            max_iter=10, q_init=q0, t_init=t0)
        assert int(res["ncorr"][0]) == c, k
        nl = int(res["nlog"][0])
        assert nl == log.shape[0], k
        glog = res["log"][0, :nl].cpu().numpy()
        for i in range(nl):
            assert np.abs(glog[i, 4:7] - log[i, 4:7]).max() < TOL_T, (k, i)
            assert _angle(glog[i, :4], log[i, :4]) < TOL_R, (k, i)
        got = rel[0].cpu().numpy()
        assert np.abs(got[4:] - t).max() < TOL_T and _angle(got[:4], q) < TOL_R, k
        q_abs, t_abs = oracle.accumulate(q_abs, t_abs, got[:4], got[4:])
        ga = ab[0].cpu().numpy()
        assert np.abs(ga[4:] - t_abs).max() < 1e-9 and np.abs(ga[:4] - q_abs).max() < 1e-12, k
    # the synthetic ego motion is ~1 m / frame forward: 32 pairs travel ~32 m
    assert 25.0 < np.linalg.norm(ab[0, 4:].cpu().numpy()) < 40.0


def test_register_chain_matches_pairwise_calls(oracle, dev):
    """ssf_register_chain (a sequence's pairs in one call, each warm start read from the previous
    pair's output slot) == one ssf_register_batch call per pair with the warm start copied in,
    bit for bit (poses, accumulated poses, correspondence counts); a frame of <= 10 plane points
    skips its pair as the reference does (:158) and the chain carries the warm start across it;
    and the chain's poses vs the oracle's chained register_pair."""
    import ssf
    F = 9
    clouds = [frame(3, k, n_az=1875)[0] for k in range(F)]
    pts = torch.from_numpy(np.concatenate(clouds)).to(dev)
    off, h_off = ssf.frame_offsets([c.shape[0] for c in clouds], dev)
    fe = ssf.Frontend(64, device=dev.index or 0, solver="gn", max_iter=10)
    pb = fe.extract_planes_batch(pts, off, h_off)
    table = fe.plane_table(pb)
    cnt = pb.count.clone()
    cnt[5] = 7                                   # frame 5: too few plane points to be a last frame
    pbk = ssf.PlaneBatch(pb.xyzi, cnt, pb.off, pb.h_off, pb.max_points)
    q0 = np.array([0.0, 0.0, 0.002, 1.0]); q0 /= np.linalg.norm(q0)
    init = torch.tensor([[*q0, 0.8, 0.02, 0.0]], dtype=torch.float64, device=dev)
    abs0 = ssf.identity_poses(1, dev)
    ch = fe.register_chain(pbk, table, init, pose_abs_init=abs0, want_ncorr=True)
    torch.cuda.synchronize()
    assert ch["pose_seq"].shape == (F - 1, 7) and ch["pose_abs_seq"].shape == (F - 1, 7)
    rel, ab = init.clone(), abs0.clone()
    seq, aseq, nc = [], [], []
    for k in range(F - 1):
        last, curr = _pair(pbk, k, k + 1)
        res = fe.register(last, table, curr, rel, ab)
        seq.append(rel.clone()); aseq.append(ab.clone()); nc.append(res["ncorr"].clone())
    torch.cuda.synchronize()
    seq = torch.cat(seq).cpu().numpy(); aseq = torch.cat(aseq).cpu().numpy()
    nc = torch.cat(nc).cpu().numpy()
    assert np.array_equal(ch["pose_seq"].cpu().numpy().view(np.uint64), seq.view(np.uint64))
    assert np.array_equal(ch["pose_abs_seq"].cpu().numpy().view(np.uint64), aseq.view(np.uint64))
    assert np.array_equal(ch["ncorr"].cpu().numpy(), nc)
    assert nc[5] == -1 and np.array_equal(seq[5], seq[4])         # the skipped pair keeps its warm start
    # vs the oracle, chained the same way
    h = pbk.count.cpu().numpy()
    planes = [pb.frame(k).cpu().numpy()[:h[k]] for k in range(F)]
    qw, tw = q0, np.array([0.8, 0.02, 0.0])
    got = ch["pose_seq"].cpu().numpy()
    for k in range(F - 1):
        q, t, _, c = oracle.register_pair(planes[k], planes[k + 1], 0.05, mode=oracle.MODE_GN,
                                          max_iter=10, q_init=qw, t_init=tw)
        assert (c if len(planes[k]) > 10 else -1) == nc[k], k
        if k != 4:          # pair 4's curr frame is the truncated one: 7 residuals for 6 DoF, an
            # ill-conditioned GN path (the chain-vs-pairwise bit equality above covers it)
            assert np.abs(got[k, 4:] - t).max() < TOL_T and _angle(got[k, :4], q) < TOL_R, k
        qw, tw = got[k, :4], got[k, 4:]
    # no pairs: nothing to do, nothing written
    one = ssf.PlaneBatch(pb.xyzi, pb.count[:1], pb.off[:2], pb.h_off[:2], pb.max_points)
    assert fe.register_chain(one, table, init)["pose_seq"].shape == (0, 7)


@pytest.fixture(scope="module")
def c4_frames():
    return [frame(9, k, n_az=4000) for k in range(2)]


def test_config4_256k_features_and_table(oracle, dev, c4_frames):
    import ssf
    fe = ssf.Frontend(64, device=dev.index or 0)
    clouds = [f[0] for f in c4_frames]
    assert clouds[0].shape[0] == 256000
    pts = torch.from_numpy(np.concatenate(clouds)).to(dev)
    off, h_off = ssf.frame_offsets([c.shape[0] for c in clouds], dev)
    pb, ring, roff, curv = fe.extract_planes_batch(pts, off, h_off, debug=True)
    normal, valid, sx, si = fe.plane_table(pb)
    torch.cuda.synchronize()
    for f, c in enumerate(clouds):
        rx, off_ref, _, _ = oracle.bin_rings(c, 64)
        cv_ref = oracle.curvature(rx, off_ref, 64)
        pl_ref, _ = oracle.select(rx, cv_ref, off_ref, 64)
        o = int(h_off[f])
        kept = int(off_ref[-1])
        assert np.array_equal(roff[f].cpu().numpy().astype(np.int64), off_ref)
        assert np.array_equal(ring[o:o + kept].cpu().numpy(), rx)
        assert np.array_equal(curv[o:o + kept].cpu().numpy().view(np.uint32), cv_ref.view(np.uint32))
        P = pb.frame(f).cpu().numpy()
        assert np.array_equal(P, pl_ref)
        assert len(P) > 6144, len(P)            # above the association's LDS staging size
        nr, vr, _, _ = oracle.plane_table(P, 0.05)
        m = len(P)
        assert np.array_equal(valid[o:o + m].cpu().numpy(), vr.astype(np.uint8)), f
        assert np.array_equal(normal[o:o + m].cpu().numpy().view(np.uint32), nr.view(np.uint32)), f


@pytest.mark.parametrize("solver,mode,iters", [("gn", 1, 10), ("ceres_lm", 0, 8)])
def test_config4_256k_association_and_registration(oracle, dev, c4_frames, solver, mode, iters):
    import ssf
    fe = ssf.Frontend(64, device=dev.index or 0, solver=solver, max_iter=iters)
    clouds = [f[0] for f in c4_frames]
    pts = torch.from_numpy(np.concatenate(clouds)).to(dev)
    off, h_off = ssf.frame_offsets([c.shape[0] for c in clouds], dev)
    pb = fe.extract_planes_batch(pts, off, h_off)
    table = fe.plane_table(pb)
    last, curr = _pair(pb, 0, 1)
    q0 = np.array([0.0, 0.0, 0.002, 1.0]); q0 /= np.linalg.norm(q0)
    t0 = np.array([0.8, 0.01, 0.0])
    rel = torch.tensor([[*q0, *t0]], dtype=torch.float64, device=dev)
    res = fe.register(last, table, curr, rel, want_log=True, want_nn=True)
    torch.cuda.synchronize()
    L, Cc = pb.frame(0).cpu().numpy(), pb.frame(1).cpu().numpy()
    o1 = int(pb.h_off[1])
    assert np.array_equal(res["nn"][o1:o1 + len(Cc)].cpu().numpy(), oracle.correspond(L, Cc, q0, t0))
    q, t, log, c = oracle.register_pair(L, Cc, 0.05, mode=mode, max_iter=iters, q_init=q0, t_init=t0)
    assert int(res["ncorr"][0]) == c
    nl = int(res["nlog"][0])
    assert nl == log.shape[0]
    glog = res["log"][0, :nl].cpu().numpy()
    for i in range(nl):
        assert glog[i, 8] == log[i, 8], i
        assert np.abs(glog[i, 4:7] - log[i, 4:7]).max() < TOL_T, i
        assert _angle(glog[i, :4], log[i, :4]) < TOL_R, i
    got = rel[0].cpu().numpy()
    assert np.abs(got[4:] - t).max() < TOL_T and _angle(got[:4], q) < TOL_R


def test_config4_256k_mask_and_kabsch(oracle, dev, c4_frames):
    import ssf
    fe = ssf.Frontend(64, device=dev.index or 0)
    pos, flow, _ = c4_frames[0]
    p = torch.from_numpy(pos).to(dev)
    fl = torch.from_numpy(flow).to(dev)
    off, h_off = ssf.frame_offsets([len(pos)], dev)
    draws = np.array([[0.25, 0.5, 0.75]])
    out, bg = fe.mask_pose(p, fl, off, h_off, mode="gmm", draws=draws)
    torch.cuda.synchronize()
    ref = oracle.mask_and_pose(pos, flow, draws[0])
    o = out[0].cpu().numpy()
    assert ref["rc"] == 0 and int(o[16]) == 0
    assert (bg.cpu().numpy() == ref["bg_mask"]).mean() >= 0.999
    assert int(o[19]) == int(ref["info"]["kmeans_iter"]) and int(o[20]) == int(ref["info"]["em_iter"])
    assert np.abs(o[0:3] - ref["t"]).max() < TOL_T and _angle(o[3:7], ref["q_xyzw"]) < TOL_R
