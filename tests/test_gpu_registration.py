"""lidarOdometry_onlyPC parity: HIP plane table / association / Ceres-LM and GN solve vs the
CPU oracle.

Bars: plane normals + validity bit-exact (same float QR sequence), 1-NN indices exact,
per-iteration poses within 1e-5 m / 1e-6 rad of the oracle (f64 reductions in a different
order), final pose likewise.
"""
import numpy as np
import pytest
import torch

from helpers import frame

pytestmark = pytest.mark.gpu

TOL_T = 1e-5   # m   (BASELINE north_star)
TOL_R = 1e-6   # rad


def _quat_angle(q1, q2):
    d = abs(float(np.dot(q1 / np.linalg.norm(q1), q2 / np.linalg.norm(q2))))
    return 2.0 * np.arccos(min(1.0, d))


def _planes(fe, dev, clouds):
    import ssf
    pts = torch.from_numpy(np.concatenate(clouds)).to(dev)
    off, h_off = ssf.frame_offsets([c.shape[0] for c in clouds], dev)
    return fe.extract_planes_batch(pts, off, h_off)


def _sub(pb, idx):
    import ssf
    # per-pair start offsets + counts into the shared plane buffer; the last entry bounds the
    # extent of the point-shaped scratch (frames are selected in ascending order)
    starts = torch.stack([pb.off[i] for i in idx])
    ends = torch.stack([pb.off[i + 1] for i in idx])
    h_st = torch.tensor([int(pb.h_off[i]) for i in idx] + [int(pb.h_off[idx[-1] + 1])])
    o = torch.cat([starts, ends[-1:]]).contiguous()
    return ssf.PlaneBatch(pb.xyzi, pb.count[idx].contiguous(), o, h_st, pb.max_points)


@pytest.mark.parametrize("brute", [False, True])
def test_plane_table_bitexact(oracle, dev, brute):
    """x-sorted walk (default) and brute-force k-NN both reproduce the oracle bit for bit"""
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    clouds = [frame(0, 0)[0], frame(1, 1)[0], frame(2, 2, n_az=1875)[0]]
    pb = _planes(fe, dev, clouds)
    normal, valid, sx, si = fe.plane_table(pb, brute_force=brute)
    if not brute:
        for f in range(3):
            o, m = int(pb.h_off[f]), int(pb.count[f])
            perm = si[o:o + m].cpu().numpy()
            xs = sx[o:o + m, 0].cpu().numpy()
            assert np.all(np.diff(xs) >= 0) and sorted(perm.tolist()) == list(range(m))
            assert np.array_equal(sx[o:o + m].cpu().numpy(), pb.frame(f).cpu().numpy()[perm])
    for f in range(3):
        P = pb.frame(f).cpu().numpy()
        nr, vr, _, _ = oracle.plane_table(P, 0.05)
        o, m = int(pb.h_off[f]), P.shape[0]
        assert np.array_equal(valid[o:o + m].cpu().numpy(), vr.astype(np.uint8))
        g = normal[o:o + m].cpu().numpy()
        assert np.array_equal(g.view(np.uint32), nr.view(np.uint32)), "normal bits differ"
        assert vr.mean() > 0.3


def test_plane_table_duplicates_and_sizes(oracle, dev):
    """Exact duplicate points (zero-distance ties broken by index) and every walk tier of the
    sorted table: points staged in LDS as 16-B records (<= 6144), as 14-B SoA arrays (<= 9088,
    with and without duplicates), read from the sorted copy in global memory (<= 16384), and
    above the LDS sort limit (brute-force k-NN) -- all bit-exact against the oracle."""
    import ssf
    rng = np.random.default_rng(7)
    base = [oracle.extract_planes(frame(s, 0, n_az=1875)[0], 64) for s in range(5)]
    dup = np.concatenate([base[0], base[0][rng.choice(len(base[0]), 600, replace=False)]])
    two = np.concatenate(base[:2])
    dup2 = np.concatenate([two, two[rng.choice(len(two), 900, replace=False)]])
    clouds = [dup[rng.permutation(len(dup))], two, dup2[rng.permutation(len(dup2))],
              np.concatenate(base[:3]), np.concatenate(base)]
    sizes = [len(c) for c in clouds]
    assert sizes[0] <= 6144 < sizes[1] < sizes[2] <= 9088 < sizes[3] <= 16384 < sizes[4], sizes
    fe = ssf.Frontend(64, device=dev.index)
    for f, P in enumerate(clouds):          # one launch each: the kernel choice is per launch
        off, h_off = ssf.frame_offsets([len(P)], dev)
        xyzi = torch.from_numpy(P.astype(np.float32)).to(dev)
        pb = ssf.PlaneBatch(xyzi, torch.tensor([len(P)], dtype=torch.int32, device=dev), off, h_off, len(P))
        normal, valid, _, _ = fe.plane_table(pb)
        nr, vr, _, _ = oracle.plane_table(P, 0.05)
        assert np.array_equal(valid.cpu().numpy(), vr.astype(np.uint8)), f
        g = normal.cpu().numpy()
        assert np.array_equal(g.view(np.uint32), nr.view(np.uint32)), f


def _rank_walk_cloud(oracle):
    """A realistic plane cloud plus an isolated dense segment of ring 20 (48 points 1 cm apart)
    with three points of rings 21 / 22 0.6-0.8 m beside it."""
    base = oracle.extract_planes(frame(0, 0)[0], 64)
    k = np.arange(48, dtype=np.float64)
    seg = np.stack([200.0 + 0.01 * k, 200.0 + 0.002 * k, 0.3 + 1e-4 * k * k, k + 0.20], 1)
    oth = np.array([[200.20, 200.60, 0.30, 3 + 0.21], [200.30, 200.70, 0.35, 4 + 0.21],
                    [200.10, 200.80, 0.32, 5 + 0.22]])
    return np.concatenate([base, seg, oth]).astype(np.float32), len(base)


def test_plane_table_rank_walk_cases(oracle, dev):
    """Queries whose first other-ring point D1 ranks beyond 30 behind many same-ring neighbours:
    the count of non-other-ring keys that left the top five exceeds the skip bound (round 6), so
    the D1 / D2 rank walk runs and decides them -- bit-exact against the oracle, as the rest of
    the frame that takes the skip."""
    import ssf
    P, nb = _rank_walk_cloud(oracle)
    # the scenario: for the segment's queries, the nearest other-ring point within 1 m ranks >= 30
    Q = P[nb:nb + 48, :3].astype(np.float64)
    rows = np.floor(100.0 * ((P[:, 3] - np.floor(P[:, 3])) + 0.002)).astype(int)
    d = np.linalg.norm(P[None, :, :3].astype(np.float64) - Q[:, None, :], axis=2)
    for j in range(48):
        order = np.argsort(d[j], kind="stable")
        ranks = [r for r, i in enumerate(order) if rows[i] != 20 and d[j, i] < 1.0]
        assert ranks and ranks[0] >= 30, (j, ranks[:3])
    fe = ssf.Frontend(64, device=dev.index)
    off, h_off = ssf.frame_offsets([len(P)], dev)
    xyzi = torch.from_numpy(P).to(dev)
    pb = ssf.PlaneBatch(xyzi, torch.tensor([len(P)], dtype=torch.int32, device=dev), off, h_off, len(P))
    normal, valid, _, _ = fe.plane_table(pb)
    nr, vr, _, _ = oracle.plane_table(P, 0.05)
    assert np.array_equal(valid.cpu().numpy(), vr.astype(np.uint8))
    g = normal.cpu().numpy()
    assert np.array_equal(g.view(np.uint32), nr.view(np.uint32)), "normal bits differ"


def test_nan_warm_start_association_stays_in_frame(dev):
    """A NaN warm start (an ill-conditioned link of a chain) makes every query point NaN: no
    candidate wins.  Both association modes -- the group mode of launches of <= 16 pairs and the
    lane mode of big launches -- fall back to the last frame's first staged point (the
    group mode used index -1, reading the neighbouring frame's records), and the call returns."""
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    clouds = [frame(0, 2, n_az=600)[0], frame(0, 3, n_az=600)[0]]
    pb = _planes(fe, dev, clouds)
    table = fe.plane_table(pb)
    m_last = int(pb.count[0])
    o1, m1 = int(pb.h_off[1]), int(pb.count[1])
    got = []
    for n_pairs in (1, 20):
        last, curr = _sub(pb, [0] * n_pairs), _sub(pb, [1] * n_pairs)
        pose = torch.full((n_pairs, 7), float("nan"), dtype=torch.float64, device=dev)
        res = fe.register(last, table, curr, pose, want_nn=True)
        torch.cuda.synchronize()
        got.append(res["nn"][o1:o1 + m1].cpu().numpy())
    for nn in got:
        assert m1 > 0 and np.all(nn == nn[0]) and 0 <= nn[0] < m_last, (np.unique(nn), m_last)
    assert np.array_equal(got[0], got[1])


@pytest.mark.parametrize("solver,iters", [("gn", 10), ("ceres_lm", 8)])
def test_compacted_records_same_bits(dev, solver, iters):
    """Big launches (> 16 pairs, one association work-group per pair) hand the solve compacted
    records in rank order and the solve streams them into LDS inside its first evaluation; a
    single-pair launch (group-mode association) writes records in query order and the solve
    compacts them itself.  Both feed the evaluations the same records in the same order: poses,
    per-step logs and correspondence counts must be bit-identical."""
    import ssf
    fe = ssf.Frontend(64, device=dev.index, solver=solver, max_iter=iters)
    # 17 pairs of one sequence (distinct current frames: the records live at their offsets)
    P = 17
    clouds = [frame(3, k, n_az=900)[0] for k in range(P + 1)]
    pb = _planes(fe, dev, clouds)
    table = fe.plane_table(pb)
    rng = np.random.default_rng(11)
    sel = [(k, k + 1) for k in range(P)]
    q0 = np.zeros((P, 4)); q0[:, 2] = rng.uniform(-0.003, 0.003, P); q0[:, 3] = 1.0
    q0 /= np.linalg.norm(q0, axis=1, keepdims=True)
    t0 = np.c_[rng.uniform(0.6, 1.1, P), rng.uniform(-0.05, 0.05, P), np.zeros(P)]
    init = torch.tensor(np.c_[q0, t0], dtype=torch.float64, device=dev)

    def sub_pairs(idx):
        import ssf as S
        lo = torch.stack([pb.off[a] for a, _ in idx] + [pb.off[idx[-1][0] + 1]])
        co = torch.stack([pb.off[b] for _, b in idx] + [pb.off[idx[-1][1] + 1]])
        hl = torch.tensor([int(pb.h_off[a]) for a, _ in idx] + [int(pb.h_off[idx[-1][0] + 1])])
        hc = torch.tensor([int(pb.h_off[b]) for _, b in idx] + [int(pb.h_off[idx[-1][1] + 1])])
        cl = torch.stack([pb.count[a] for a, _ in idx]).contiguous()
        cc = torch.stack([pb.count[b] for _, b in idx]).contiguous()
        return (S.PlaneBatch(pb.xyzi, cl, lo.contiguous(), hl, pb.max_points),
                S.PlaneBatch(pb.xyzi, cc, co.contiguous(), hc, pb.max_points))

    last, curr = sub_pairs(sel)
    big = fe.register(last, table, curr, init.clone(), want_log=True)
    torch.cuda.synchronize()
    for k in range(P):
        l1, c1 = sub_pairs([sel[k]])
        one = fe.register(l1, table, c1, init[k:k + 1].clone(), want_log=True)
        torch.cuda.synchronize()
        assert int(one["ncorr"][0]) == int(big["ncorr"][k]) > 0
        assert np.array_equal(one["pose_rel"][0].cpu().numpy().view(np.uint64),
                              big["pose_rel"][k].cpu().numpy().view(np.uint64)), k
        n = int(one["nlog"][0])
        assert n == int(big["nlog"][k])
        assert np.array_equal(one["log"][0, :n].cpu().numpy().view(np.uint64),
                              big["log"][k, :n].cpu().numpy().view(np.uint64)), k


def test_compacted_records_edge_pairs(dev):
    """The compacted-record path's edge cases inside one big launch (> 16 pairs): a pair whose
    last frame has <= 10 plane points (:158, skipped, count 0), a pair with an empty current
    frame, and a pair whose current frame is cut to 3 points -- every pair's pose, log and count
    bit-identical to its own single-pair launch (group-mode association, solve-side compaction)."""
    import ssf
    fe = ssf.Frontend(64, device=dev.index, solver="gn", max_iter=10)
    P = 18
    clouds = [frame(4, k, n_az=900)[0] for k in range(P + 1)]
    pb = _planes(fe, dev, clouds)
    table = fe.plane_table(pb)
    init = torch.tensor([[0.0, 0.0, 0.001, 1.0, 0.8, 0.0, 0.0]] * P, dtype=torch.float64, device=dev)
    init[:, :4] /= torch.linalg.norm(init[:, :4], dim=1, keepdim=True)
    cut_last = {2: 8, 9: 10}                   # last-frame plane counts <= 10
    cut_curr = {5: 0, 13: 3}                   # an empty and a 3-point current frame

    def pairs(idx):
        lo = torch.stack([pb.off[k] for k in idx] + [pb.off[idx[-1] + 1]])
        co = torch.stack([pb.off[k + 1] for k in idx] + [pb.off[idx[-1] + 2]])
        hl = torch.tensor([int(pb.h_off[k]) for k in idx] + [int(pb.h_off[idx[-1] + 1])])
        hc = torch.tensor([int(pb.h_off[k + 1]) for k in idx] + [int(pb.h_off[idx[-1] + 2])])
        cl = torch.stack([torch.clamp(pb.count[k], max=cut_last.get(k, 1 << 30)) for k in idx]).contiguous()
        cc = torch.stack([torch.clamp(pb.count[k + 1], max=cut_curr.get(k, 1 << 30)) for k in idx]).contiguous()
        return (ssf.PlaneBatch(pb.xyzi, cl, lo.contiguous(), hl, pb.max_points),
                ssf.PlaneBatch(pb.xyzi, cc, co.contiguous(), hc, pb.max_points))

    last, curr = pairs(list(range(P)))
    big = fe.register(last, table, curr, init.clone(), want_log=True)
    torch.cuda.synchronize()
    for k in range(P):
        l1, c1 = pairs([k])
        one = fe.register(l1, table, c1, init[k:k + 1].clone(), want_log=True)
        torch.cuda.synchronize()
        assert int(one["ncorr"][0]) == int(big["ncorr"][k]), k
        assert np.array_equal(one["pose_rel"][0].cpu().numpy().view(np.uint64),
                              big["pose_rel"][k].cpu().numpy().view(np.uint64)), k
        n = int(one["nlog"][0])
        assert n == int(big["nlog"][k]), k
        assert np.array_equal(one["log"][0, :n].cpu().numpy().view(np.uint64),
                              big["log"][k, :n].cpu().numpy().view(np.uint64)), k
    for k in list(cut_last) + [5]:
        assert int(big["ncorr"][k]) <= 0, (k, int(big["ncorr"][k]))


@pytest.mark.parametrize("solver,iters,mode,brute", [("ceres_lm", 8, 0, False), ("gn", 10, 1, False),
                                                     ("ceres_lm", 8, 0, True)])
def test_register_pair_per_step(oracle, dev, solver, iters, mode, brute):
    import ssf
    fe = ssf.Frontend(64, device=dev.index, solver=solver, max_iter=iters)
    clouds = [frame(0, 2, n_az=1875)[0], frame(0, 3, n_az=1875)[0]]
    pb = _planes(fe, dev, clouds)
    table = fe.plane_table(pb, brute_force=brute)
    last, curr = _sub(pb, [0]), _sub(pb, [1])
    q0 = np.array([0.0, 0.0, 0.001, 1.0]); q0 /= np.linalg.norm(q0)
    t0 = np.array([0.9, 0.01, 0.0])
    pose = torch.tensor([[*q0, *t0]], dtype=torch.float64, device=dev)
    res = fe.register(last, table, curr, pose, want_log=True, want_nn=True)
    torch.cuda.synchronize()
    L = pb.frame(0).cpu().numpy()
    Cc = pb.frame(1).cpu().numpy()
    nn_ref = oracle.correspond(L, Cc, q0, t0)
    o1 = int(pb.h_off[1])
    assert np.array_equal(res["nn"][o1:o1 + Cc.shape[0]].cpu().numpy(), nn_ref)
    q, t, log, c = oracle.register_pair(L, Cc, 0.05, mode=mode, max_iter=iters, q_init=q0, t_init=t0)
    assert int(res["ncorr"][0]) == c
    nl = int(res["nlog"][0])
    assert nl == log.shape[0], (nl, log[:, 8])
    glog = res["log"][0, :nl].cpu().numpy()
    for k in range(nl):
        assert glog[k, 8] == log[k, 8], f"step {k} status differs"
        assert np.abs(glog[k, 4:7] - log[k, 4:7]).max() < TOL_T, k
        assert _quat_angle(glog[k, :4], log[k, :4]) < TOL_R, k
        assert abs(glog[k, 7] - log[k, 7]) <= 1e-9 * max(1.0, abs(log[k, 7]))
    got = res["pose_rel"][0].cpu().numpy()
    assert np.abs(got[4:] - t).max() < TOL_T and _quat_angle(got[:4], q) < TOL_R


def test_gn_steps_both_quaternion_update_paths(oracle, dev):
    """k_solve's GN update takes Taylor polynomials for steps theta < 2^-7 and libm sin / cos
    above (quat_plus_step): a warm start 0.05 rad off gives both kinds of step in one solve; every
    step's pose stays within the per-step bar of the oracle's (libm) update."""
    import ssf
    fe = ssf.Frontend(64, device=dev.index, solver="gn", max_iter=10)
    clouds = [frame(0, 2, n_az=1875)[0], frame(0, 3, n_az=1875)[0]]
    pb = _planes(fe, dev, clouds)
    table = fe.plane_table(pb)
    last, curr = _sub(pb, [0]), _sub(pb, [1])
    q0 = np.array([0.0, 0.0, np.sin(0.025), np.cos(0.025)])
    t0 = np.array([0.9, 0.01, 0.0])
    pose = torch.tensor([[*q0, *t0]], dtype=torch.float64, device=dev)
    res = fe.register(last, table, curr, pose, want_log=True)
    torch.cuda.synchronize()
    L = pb.frame(0).cpu().numpy()
    Cc = pb.frame(1).cpu().numpy()
    q, t, log, c = oracle.register_pair(L, Cc, 0.05, mode=1, max_iter=10, q_init=q0, t_init=t0)
    nl = int(res["nlog"][0])
    assert nl == log.shape[0]
    glog = res["log"][0, :nl].cpu().numpy()
    for k in range(nl):
        assert glog[k, 8] == log[k, 8], f"step {k} status differs"
        assert np.abs(glog[k, 4:7] - log[k, 4:7]).max() < TOL_T, k
        assert _quat_angle(glog[k, :4], log[k, :4]) < TOL_R, k
    # a step of theta turns the pose by 2 theta
    turns = [_quat_angle(log[0, :4], q0)] + [_quat_angle(log[k, :4], log[k - 1, :4]) for k in range(1, nl)]
    assert max(turns) > 2 * 2.0 ** -7 and min(turns) < 2 * 2.0 ** -7, turns
    got = res["pose_rel"][0].cpu().numpy()
    assert np.abs(got[4:] - t).max() < TOL_T and _quat_angle(got[:4], q) < TOL_R


def test_16_row_profile_table_and_registration(oracle, dev):
    """16-beam profile (planeMax 0.15, lidarOdometry_onlyPC.cpp:314-316): plane table bit-exact
    and an LM pair within the pose bars."""
    import ssf
    fe = ssf.Frontend(16, device=dev.index)
    clouds = [frame(3, 0, n_rows=16, n_az=1800)[0], frame(3, 1, n_rows=16, n_az=1800)[0]]
    pb = _planes(fe, dev, clouds)
    table = fe.plane_table(pb)
    normal, valid = table[0], table[1]
    for f in range(2):
        P = pb.frame(f).cpu().numpy()
        nr, vr, _, _ = oracle.plane_table(P, 0.15)
        o, m = int(pb.h_off[f]), P.shape[0]
        assert np.array_equal(valid[o:o + m].cpu().numpy(), vr.astype(np.uint8))
        assert np.array_equal(normal[o:o + m].cpu().numpy().view(np.uint32), nr.view(np.uint32))
    q0, t0 = np.array([0.0, 0.0, 0.0, 1.0]), np.array([0.5, 0.0, 0.0])
    pose = torch.tensor([[*q0, *t0]], dtype=torch.float64, device=dev)
    res = fe.register(_sub(pb, [0]), table, _sub(pb, [1]), pose, want_nn=True)
    torch.cuda.synchronize()
    L, Cc = pb.frame(0).cpu().numpy(), pb.frame(1).cpu().numpy()
    o1 = int(pb.h_off[1])
    assert np.array_equal(res["nn"][o1:o1 + len(Cc)].cpu().numpy(), oracle.correspond(L, Cc, q0, t0))
    q, t, _, c = oracle.register_pair(L, Cc, 0.15, mode=0, max_iter=8, q_init=q0, t_init=t0)
    got = res["pose_rel"][0].cpu().numpy()
    assert int(res["ncorr"][0]) == c
    assert np.abs(got[4:] - t).max() < TOL_T and _quat_angle(got[:4], q) < TOL_R


@pytest.mark.parametrize("k", [2, 3, 4])
def test_associate_large_frames(oracle, dev, k):
    """1-NN indices exact above the 16-B LDS staging size (6144 plane points): k = 2, 3 stage the
    last frame as 12-B SoA arrays (<= 12032, ties resolved through the global permutation), k = 4
    walks the sorted last frame in global memory.  The last frame holds exact duplicates, so
    distance ties occur and must resolve to the lower original index."""
    import ssf
    rng = np.random.default_rng(11 + k)
    base = [oracle.extract_planes(frame(s, 0, n_az=1875)[0], 64) for s in range(k + 1)]
    L = np.concatenate(base[:k])
    L = np.concatenate([L, L[rng.choice(len(L), 300, replace=False)]])
    L = L[rng.permutation(len(L))]
    Cc = np.concatenate(base[1:])
    assert 6144 < len(L) and (len(L) <= 12032) == (k < 4) and len(L) <= 16384
    fe = ssf.Frontend(64, device=dev.index)
    sizes = [len(L), len(Cc)]
    off, h_off = ssf.frame_offsets(sizes, dev)
    xyzi = torch.from_numpy(np.concatenate([L, Cc]).astype(np.float32)).to(dev)
    pb = ssf.PlaneBatch(xyzi, torch.tensor(sizes, dtype=torch.int32, device=dev), off, h_off, max(sizes))
    table = fe.plane_table(pb)
    q0 = np.array([0.0, 0.0, 0.002, 1.0]); q0 /= np.linalg.norm(q0)
    t0 = np.array([0.5, -0.02, 0.01])
    pose = torch.tensor([[*q0, *t0]], dtype=torch.float64, device=dev)
    res = fe.register(_sub(pb, [0]), table, _sub(pb, [1]), pose, want_nn=True)
    torch.cuda.synchronize()
    o1 = int(h_off[1])
    assert np.array_equal(res["nn"][o1:o1 + len(Cc)].cpu().numpy(), oracle.correspond(L, Cc, q0, t0))


def test_register_batch_and_accumulate(oracle, dev):
    """3 independent pairs in one launch + pose accumulation (publishResult :87-90); one pair
    whose last frame has <= 10 plane points is skipped (:158) and keeps its warm start."""
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    c = frame(3, 0)[0][:64 * 12]          # 12 azimuth steps of rows 5..12 -> 8 plane points
    r = np.arange(c.shape[0]) % 64
    tiny = c[(r >= 5) & (r < 13)]
    clouds = [frame(1, 0)[0], frame(1, 1)[0], frame(2, 4)[0], frame(2, 5)[0], tiny, frame(3, 1)[0]]
    pb = _planes(fe, dev, clouds)
    table = fe.plane_table(pb)
    last, curr = _sub(pb, [0, 2, 4]), _sub(pb, [1, 3, 5])
    rel = ssf.identity_poses(3, dev)
    rel[2, 4] = 0.5
    ab = ssf.identity_poses(3, dev)
    ab[:, 4] = 10.0
    res = fe.register(last, table, curr, rel, ab)
    torch.cuda.synchronize()
    for p, (a, b) in enumerate([(0, 1), (2, 3), (4, 5)]):
        L, Cc = pb.frame(a).cpu().numpy(), pb.frame(b).cpu().numpy()
        qi = [0, 0, 0, 1]; ti = [0.5 if p == 2 else 0.0, 0, 0]
        q, t, log, c = oracle.register_pair(L, Cc, 0.05, q_init=qi, t_init=ti)
        got = rel[p].cpu().numpy()
        assert int(res["ncorr"][p]) == c
        assert np.abs(got[4:] - t).max() < TOL_T and _quat_angle(got[:4], q) < TOL_R
        qa, ta = oracle.accumulate([0, 0, 0, 1], [10.0, 0, 0], q, t)
        ga = ab[p].cpu().numpy()
        assert np.abs(ga[4:] - ta).max() < TOL_T and _quat_angle(ga[:4], qa) < TOL_R
    assert pb.count[4].item() <= 10 and int(res["ncorr"][2]) == -1


def test_accumulate_sequence(oracle, dev):
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    rng = np.random.default_rng(0)
    rel = np.zeros((20, 7))
    for i in range(20):
        q = rng.normal(0, 0.01, 4); q[3] = 1.0; q /= np.linalg.norm(q)
        rel[i, :4] = q; rel[i, 4:] = rng.normal(0, 1, 3)
    out = fe.accumulate_sequence(torch.tensor(rel, device=dev)).cpu().numpy()
    q, t = np.array([0, 0, 0, 1.0]), np.zeros(3)
    for i in range(20):
        q, t = oracle.accumulate(q, t, rel[i, :4], rel[i, 4:])
        assert np.abs(out[i, 4:] - t).max() < 1e-12 and np.abs(out[i, :4] - q).max() < 1e-12


@pytest.mark.parametrize("solver,iters,mode", [("ceres_lm", 8, 0), ("gn", 10, 1)])
def test_ssf_register_pair_abi(oracle, dev, solver, iters, mode):
    """ssf_register_pair: frameRegistration() on the reference's globals --
    raw last/current plane clouds, para_q/para_t warm start in, solution + per-step log out
    (lidarOdometry_onlyPC.cpp:147-252).  Per-iteration poses, costs and status codes against the
    oracle; the warm start is chained over three consecutive pairs as cloudThread does
    (:251-252, :307)."""
    import ssf
    fe = ssf.Frontend(64, device=dev.index, solver=solver, max_iter=iters)
    planes = [oracle.extract_planes(frame(4, k, n_az=1875)[0], 64) for k in range(4)]
    q, t = [0.0, 0.0, 0.0, 1.0], [0.0, 0.0, 0.0]
    qr, tr = np.array(q), np.array(t)
    for k in range(1, 4):
        L = torch.from_numpy(planes[k - 1]).to(dev)
        Cc = torch.from_numpy(planes[k]).to(dev)
        q, t, steps, nc = fe.register_pair(L, Cc, q, t)
        qr, tr, log, c = oracle.register_pair(planes[k - 1], planes[k], 0.05, mode=mode,
                                              max_iter=iters, q_init=qr, t_init=tr)
        assert nc == c and len(steps) == log.shape[0], (k, nc, c, len(steps), log.shape)
        for i, st in enumerate(steps):
            assert ssf._abi.STEP_STATUS[int(log[i, 8])] == st["status"], (k, i)
            assert np.abs(np.array(st["t"]) - log[i, 4:7]).max() < TOL_T, (k, i)
            assert _quat_angle(np.array(st["q"]), log[i, :4]) < TOL_R, (k, i)
            assert abs(st["cost"] - log[i, 7]) <= 1e-9 * max(1.0, abs(log[i, 7]))
        assert np.abs(np.array(t) - tr).max() < TOL_T and _quat_angle(np.array(q), qr) < TOL_R
        qr, tr = np.array(q), np.array(t)       # chain the GPU solution (bars are per pair)


def test_ssf_register_pair_skip_and_empty(dev):
    """<= 10 last-frame points: no residual, the warm start is returned unchanged (:158)."""
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    small = torch.zeros((10, 4), dtype=torch.float32, device=dev)
    curr = torch.from_numpy(np.random.default_rng(0).normal(size=(50, 4)).astype(np.float32)).to(dev)
    q0, t0 = [0.0, 0.0, 0.1, 0.99498743710662], [0.5, 0.25, -0.125]
    q, t, steps, nc = fe.register_pair(small, curr, q0, t0)
    assert q == q0 and t == t0 and steps == [] and nc == -1
    empty = torch.zeros((0, 4), dtype=torch.float32, device=dev)
    q, t, steps, nc = fe.register_pair(curr, empty, q0, t0)
    assert q == q0 and t == t0 and nc == 0


@pytest.mark.parametrize("n_pairs", [1, 3])
def test_strip_image_reuse_identical(dev, n_pairs):
    """The association staging the plane table's strip image (PlaneTable.strips) answers exactly
    as the one building its own strips: identical 1-NN indices, correspondence counts and pose
    bits, for one pair (8 work-groups per pair) and several, with a last frame below the image's
    773-point minimum (rebuilt) in the same launch."""
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    full = [frame(s, 4 + s, n_az=1875)[0] for s in range(n_pairs)]
    nxt = [frame(s, 5 + s, n_az=1875)[0] for s in range(n_pairs)]
    pb = _planes(fe, dev, full + nxt)
    if n_pairs > 1:                                   # pair 0's last frame: a 600-point cut
        P0 = pb.frame(0)[:600].clone()
        rest = [pb.frame(f) for f in range(1, 2 * n_pairs)]
        xyzi = torch.cat([P0, *rest]).contiguous()
        counts = [600] + [int(r.shape[0]) for r in rest]
        off, h_off = ssf.frame_offsets(counts, dev)
        pb = ssf.PlaneBatch(xyzi, torch.tensor(counts, dtype=torch.int32, device=dev), off, h_off,
                            max(counts))
    m = [int(c) for c in pb.count.cpu()]
    assert any(773 <= c <= 6144 for c in m[:n_pairs]), m
    t_img = fe.plane_table(pb)
    t_new = fe.plane_table(pb, strips=False)
    assert t_img.strips is not None and t_new.strips is None
    last, curr = _sub(pb, list(range(n_pairs))), _sub(pb, list(range(n_pairs, 2 * n_pairs)))
    q0 = np.array([0.0, 0.0, 0.002, 1.0]); q0 /= np.linalg.norm(q0)
    pose0 = torch.tensor([[*q0, 0.8, 0.02, 0.0]] * n_pairs, dtype=torch.float64, device=dev)
    out = []
    for tb in (t_img, t_new):
        pose = pose0.clone()
        r = fe.register(last, tb, curr, pose, want_nn=True)
        torch.cuda.synchronize()
        out.append((r["nn"].cpu().numpy(), r["ncorr"].cpu().numpy(), r["pose_rel"].cpu().numpy()))
    assert np.array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1])
    assert np.array_equal(out[0][2].view(np.uint64), out[1][2].view(np.uint64))


def test_strip_image_argument_checks(dev):
    """The strip image travels as a pair (image and header) and only with the sorted buffers:
    anything else is SSF_E_ARG with a message, before any launch."""
    import ssf
    from ssf import _abi
    from ssf.frontend import _ptr, _stream
    fe = ssf.Frontend(64, device=dev.index)
    pb = _planes(fe, dev, [frame(0, 6, n_az=1875)[0]])
    total = pb.xyzi.shape[0]
    t = lambda *shape, dt=torch.float32: torch.empty(shape, dtype=dt, device=dev)  # noqa: E731
    normal, valid = t(total, 3), t(total, dt=torch.uint8)
    sx, si, img, head = t(total, 4), t(total, dt=torch.int32), t(total, 4), t(total, dt=torch.int32)
    L = _abi.lib()
    base = (fe._h, _stream(dev), 1, _ptr(pb.xyzi), _ptr(pb.off), _ptr(pb.count), pb.max_points,
            _ptr(normal), _ptr(valid))
    for args in ((_ptr(sx), _ptr(si), _ptr(img), None), (_ptr(sx), _ptr(si), None, _ptr(head)),
                 (None, None, _ptr(img), _ptr(head))):
        assert L.ssf_plane_table_batch(*base, *args) != 0
        assert b"strip image" in L.ssf_last_error(fe._h)
    assert L.ssf_plane_table_batch(*base, _ptr(sx), _ptr(si), _ptr(img), _ptr(head)) == 0
    torch.cuda.synchronize()


def test_kabsch_warm_start_independent_pairs(oracle, dev):
    """bench.py --kabsch-warm-start (beyond the reference): every pair of a
    sequence warm-started from its own SSF Kabsch pose (mask_and_pose of its last frame, whose
    flow points into the next frame), all pairs in ONE register launch -- each pair equals
    oracle.register_pair with the same warm start (GN x 10, per-pair poses within the bars)."""
    import ssf
    fe = ssf.Frontend(64, device=dev.index, solver="gn", max_iter=10)
    F = 4
    fr = [frame(5, k, n_az=1875) for k in range(F)]
    pb = _planes(fe, dev, [f[0] for f in fr])
    table = fe.plane_table(pb)
    # the SSF poses of frames 0..F-2 (T_{k <- k+1}) in one mask launch
    P = np.concatenate([f[0] for f in fr[:-1]]); Fl = np.concatenate([f[1] for f in fr[:-1]])
    mp = ssf.mask_and_pose(P, Fl, mode="gt", gt_mask=np.concatenate([f[2] for f in fr[:-1]]),
                           frame_sizes=[len(f[0]) for f in fr[:-1]])
    ws = np.concatenate([mp["q_xyzw"], mp["t"]], 1)                      # [F-1, 7] (q, t)
    pose = torch.from_numpy(ws.copy()).to(dev)
    last, curr = _sub(pb, list(range(F - 1))), _sub(pb, list(range(1, F)))
    res = fe.register(last, table, curr, pose)
    torch.cuda.synchronize()
    got = res["pose_rel"].cpu().numpy()
    for p in range(F - 1):
        L, Cc = pb.frame(p).cpu().numpy(), pb.frame(p + 1).cpu().numpy()
        q, t, _, c = oracle.register_pair(L, Cc, 0.05, mode=1, max_iter=10, q_init=ws[p, :4], t_init=ws[p, 4:])
        assert int(res["ncorr"][p]) == c
        assert np.abs(got[p, 4:] - t).max() < TOL_T and _quat_angle(got[p, :4], q) < TOL_R, p
        # the warm start is already close: the registration moves it by decimetres at most
        assert np.abs(got[p, 4:] - ws[p, 4:]).max() < 0.2


def test_strip_image_invalidated_when_not_imaged(dev):
    """a plane-table launch that does not image its frames (here the brute-force table,
    max_plane_points above the sort limit) clears their header's validity word, so an association
    handed these strip buffers rebuilds its strips instead of reading a stale image."""
    import ssf
    from ssf import _abi
    from ssf.frontend import _ptr, _stream
    fe = ssf.Frontend(64, device=dev.index)
    pb = _planes(fe, dev, [frame(3, 1, n_az=1875)[0], frame(3, 2, n_az=1875)[0]])
    m = [int(c) for c in pb.count.cpu()]
    assert all(_abi.STRIP_IMAGE_MIN <= c <= _abi.STRIP_IMAGE_MAX for c in m), m
    total = pb.xyzi.shape[0]
    normal = torch.empty((total, 3), dtype=torch.float32, device=dev)
    valid = torch.empty(total, dtype=torch.uint8, device=dev)
    sx = torch.empty((total, 4), dtype=torch.float32, device=dev)
    si = torch.empty(total, dtype=torch.int32, device=dev)
    img = torch.zeros((total, 4), dtype=torch.float32, device=dev)
    head = torch.zeros(total, dtype=torch.int32, device=dev)
    word = 3 * 256 + 4                                  # ns | magic << 16
    offs = [int(v) for v in pb.h_off[:2]]
    for o in offs:
        head[o + word] = 0x57A1 << 16 | 7               # a stale "valid" header
    rc = _abi.lib().ssf_plane_table_batch(fe._h, _stream(dev), 2, _ptr(pb.xyzi), _ptr(pb.off),
                                          _ptr(pb.count), 20000, _ptr(normal), _ptr(valid), _ptr(sx),
                                          _ptr(si), _ptr(img), _ptr(head))
    assert rc == 0
    torch.cuda.synchronize()
    assert [int(head[o + word]) for o in offs] == [0, 0]
    t = fe.plane_table(pb)                              # the sorted table images them again
    torch.cuda.synchronize()
    assert all((int(t.strips[1][o + word]) >> 16) == 0x57A1 for o in offs)


def test_plane_table_split_over_work_groups(oracle, dev):
    """Small batches split a frame's queries over up to 8 work-groups (launch_plane_table:
    min(8, 256 / frames, m / 256) shares, each sorting and building the strips itself): the same
    frame in batches of 1, 5, 40 and 256 frames (8, 8, 6 and 1 shares) gives bit-identical
    normals, validity, sorted copy and strip image, equal to the oracle"""
    import ssf
    c = frame(3, 4, n_az=1875)[0]
    ref = None
    for B in (1, 5, 40, 256):
        fe = ssf.Frontend(64, device=dev.index or 0)
        pb = _planes(fe, dev, [c] * B)
        tab = fe.plane_table(pb)
        normal, valid, sx, si = tab
        o, m = int(pb.h_off[B - 1]), int(pb.count[B - 1])
        got = [normal[o:o + m].cpu().numpy().view(np.uint32), valid[o:o + m].cpu().numpy(),
               sx[o:o + m].cpu().numpy(), si[o:o + m].cpu().numpy()]
        if tab.strips is not None:                            # the image and its defined head words
            img, head = (t[o:o + m].cpu().numpy() for t in tab.strips)
            K = 256                                           # kStripMax (registration.hip)
            ns = int(head[3 * K + 4]) & 0xFFFF
            got += [img, head[:K + 1], head[K + 1:K + 1 + ns], head[2 * K + 1:2 * K + 1 + ns],
                    head[3 * K + 1:3 * K + 5]]
        if ref is None:
            ref = got
            nr, vr, _, _ = oracle.plane_table(pb.frame(0).cpu().numpy(), 0.05)
            assert np.array_equal(got[0], nr.view(np.uint32)), "normal bits differ"
            assert np.array_equal(got[1], vr.astype(np.uint8))
        assert len(got) == len(ref), B
        for a, b in zip(got, ref):
            assert np.array_equal(a, b), B


def test_plane_table_split_global_deferred_walk(oracle, dev):
    """with the queries of one frame split over several work-groups, the
    strip-walk tier's deferred queries read the sorted copy back from global memory
    (table_deferred_walk: a full queue, or a query still undecided after the 6 m strips).  Every
    share must read its OWN copy.  Frames that take that tier at B = 1 (8 shares): a sparse
    frame whose 30-NN reach far beyond 6 m with ring codes the list-free pick cannot use
    (negative intensities), and a 14-B SoA frame (9217..10624 points).  The caching allocator is
    filled with NaN first so a read of unwritten memory cannot pass by luck.  Bit-exact vs the
    oracle, and equal at B = 1 and B = 256."""
    import ssf
    rng = np.random.default_rng(11)
    n = 2000
    sparse = np.zeros((n, 4), np.float32)
    sparse[:, 0] = rng.uniform(-150, 150, n)
    sparse[:, 1] = rng.uniform(-150, 150, n)
    sparse[:, 2] = rng.choice([-2.5, 0.0, 3.0], n) + rng.normal(0, 0.01, n)
    sparse[:, 3] = -(rng.integers(0, 500, n) + rng.integers(0, 64, n) / 100.0)
    base = np.concatenate([oracle.extract_planes(frame(s, 0, n_az=1875)[0], 64) for s in range(4)])
    soa = base[rng.choice(len(base), 10000, replace=False)]
    assert 9216 < len(soa) <= 10624
    for P in (sparse, soa):
        nr, vr, _, _ = oracle.plane_table(P, 0.05)
        ref = None
        for B in (1, 256):
            junk = torch.full((64 << 20,), float("nan"), device=dev)   # poison the allocator's pool
            del junk
            fe = ssf.Frontend(64, device=dev.index or 0)
            m = len(P)
            xyzi = torch.from_numpy(np.tile(P.astype(np.float32), (B, 1))).to(dev)
            off, h_off = ssf.frame_offsets([m] * B, dev)
            pb = ssf.PlaneBatch(xyzi, torch.full((B,), m, dtype=torch.int32, device=dev), off, h_off, m)
            normal, valid, sx, si = fe.plane_table(pb)
            o = int(h_off[B - 1])
            got = [normal[o:o + m].cpu().numpy().view(np.uint32), valid[o:o + m].cpu().numpy(),
                   sx[o:o + m].cpu().numpy(), si[o:o + m].cpu().numpy()]
            assert np.array_equal(got[0], nr.view(np.uint32)), (m, B, "normal bits differ")
            assert np.array_equal(got[1], vr.astype(np.uint8)), (m, B)
            if ref is None:
                ref = got
            for a, b in zip(got, ref):
                assert np.array_equal(a, b), (m, B)
