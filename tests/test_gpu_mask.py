"""Mask + Kabsch parity: the HIP GaussianMixture / slove_RT_by_SVD / quaternion block vs
(a) golden vectors generated from the reference's own PointCloudOdometry_noSeg.py + sklearn
(tests/golden/make_golden.py) and (b) the CPU oracle at the full 120k-point size.

Bars: labels identical to sklearn's on the fixtures (>= 99.9 % required, BASELINE), k-means++
centre indices and KMeans / EM iteration counts identical, R/t within 1e-5 m / 1e-6 rad
(observed ~1e-12), published [t, q] likewise.
"""
import glob
import os

import numpy as np
import pytest
import torch

from helpers import frame

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _run(fe, dev, clouds, flows, mode="gmm", mask=None, draws=None, reflection=0):
    import ssf
    pts = torch.from_numpy(np.concatenate(clouds).astype(np.float32)).to(dev)
    fl = torch.from_numpy(np.concatenate(flows).astype(np.float32)).to(dev)
    off, h_off = ssf.frame_offsets([c.shape[0] for c in clouds], dev)
    m = None if mask is None else torch.from_numpy(np.concatenate(mask).astype(np.uint8)).to(dev)
    out, bg = fe.mask_pose(pts, fl, off, h_off, mode=mode, mask_in=m, draws=draws, reflection=reflection)
    torch.cuda.synchronize()
    return out.cpu().numpy(), bg.cpu().numpy(), h_off


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "gmm_noseg_case*.npz"))))
def test_gmm_mask_vs_reference_golden(dev, path):
    import ssf
    g = np.load(path)
    fe = ssf.Frontend(64, device=dev.index)
    out, bg, _ = _run(fe, dev, [g["pos1"]], [g["flow"]], draws=g["draws"][None, :])
    o = out[0]
    assert o[16] == 0
    assert [int(o[22]), int(o[23])] == [int(v) for v in g["kmeans_pp_idx"]]
    assert int(o[19]) == int(g["kmeans_n_iter"]) and int(o[20]) == int(g["gmm_n_iter"])
    bg_ref = (g["labels"] == int(g["bg_label"])).astype(np.uint8)
    agree = (bg == bg_ref).mean()
    assert agree >= 0.999
    assert agree == 1.0
    assert abs(o[24] - float(g["gmm_lower_bound"])) < 1e-9
    assert np.abs(o[7:16].reshape(3, 3) - g["R"]).max() < 1e-6
    assert np.abs(o[0:3] - g["t"]).max() < 1e-5
    assert np.abs(np.r_[o[0:3], o[3:7]] - g["para_t_q"]).max() < 1e-6


def test_context_rng_matches_np_random_seed(dev):
    """ssf_rng_seed(s) == np.random.seed(s): frame k consumes draws 3k..3k+2"""
    import ssf
    g = np.load(os.path.join(GOLDEN, "gmm_noseg_case1.npz"))
    fe = ssf.Frontend(64, device=dev.index)
    fe.seed(int(g["seed"]))
    out, _, _ = _run(fe, dev, [g["pos1"]], [g["flow"]])
    assert [int(out[0, 22]), int(out[0, 23])] == [int(v) for v in g["kmeans_pp_idx"]]


def test_full_size_batch_vs_oracle(oracle, dev):
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    fr = [frame(5, 0, n_az=1875), frame(5, 1, n_az=1875), frame(6, 3, n_az=1875)]
    draws = np.array([[0.11, 0.52, 0.93], [0.7, 0.2, 0.4], [0.5, 0.5, 0.5]])
    out, bg, h_off = _run(fe, dev, [f[0] for f in fr], [f[1] for f in fr], draws=draws)
    for k, f in enumerate(fr):
        ref = oracle.mask_and_pose(f[0], f[1], draws[k])
        o = out[k]
        assert o[16] == ref["rc"] == 0
        assert int(o[22]) == int(ref["info"]["center0"]) and int(o[23]) == int(ref["info"]["center1"])
        a, b = int(h_off[k]), int(h_off[k + 1])
        agree = (bg[a:b] == ref["bg_mask"]).mean()
        assert agree >= 0.999, agree
        assert np.abs(o[0:3] - ref["t"]).max() < 1e-5
        assert np.abs(o[7:16].reshape(3, 3) - ref["R"]).max() < 1e-6


@pytest.mark.parametrize("G", [1, 2, 3, 5, 8])
def test_frame_split_golden(dev, G):
    """ssf_set_mask_split: the GMM fit of one frame on G work-groups exchanging per-pass sums
    (G = 1: the B >= 256 bench path; the automatic choice for a 1-frame launch is 8).  Labels,
    k-means++ indices, iteration counts and the lower bound stay those of sklearn."""
    import ssf
    g = np.load(os.path.join(GOLDEN, "gmm_noseg_case2.npz"))
    fe = ssf.Frontend(64, device=dev.index)
    fe.mask_split(G)
    out, bg, _ = _run(fe, dev, [g["pos1"]], [g["flow"]], draws=g["draws"][None, :])
    o = out[0]
    assert o[16] == 0
    assert [int(o[22]), int(o[23])] == [int(v) for v in g["kmeans_pp_idx"]]
    assert int(o[19]) == int(g["kmeans_n_iter"]) and int(o[20]) == int(g["gmm_n_iter"])
    assert np.array_equal(bg, (g["labels"] == int(g["bg_label"])).astype(np.uint8))
    assert abs(o[24] - float(g["gmm_lower_bound"])) < 1e-9
    assert np.abs(o[0:3] - g["t"]).max() < 1e-5


@pytest.mark.parametrize("G", [1, 4])
def test_frame_split_full_size_vs_oracle(oracle, dev, G):
    """120k-point frames with the split fixed at 1 and 4 parts per frame vs the oracle."""
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    fe.mask_split(G)
    fr = [frame(7, 2, n_az=1875), frame(8, 4, n_az=1875)]
    draws = np.array([[0.31, 0.62, 0.13], [0.9, 0.05, 0.45]])
    out, bg, h_off = _run(fe, dev, [f[0] for f in fr], [f[1] for f in fr], draws=draws)
    for k, f in enumerate(fr):
        ref = oracle.mask_and_pose(f[0], f[1], draws[k])
        o = out[k]
        assert o[16] == ref["rc"] == 0
        assert int(o[19]) == int(ref["info"]["kmeans_iter"]) and int(o[20]) == int(ref["info"]["em_iter"])
        a, b = int(h_off[k]), int(h_off[k + 1])
        assert (bg[a:b] == ref["bg_mask"]).mean() >= 0.999
        assert np.abs(o[0:3] - ref["t"]).max() < 1e-5


@pytest.mark.parametrize("G", [1, 2])
def test_mask_schedule_order_and_queue_same_outputs(dev, G):
    """ssf_set_mask_schedule: a dispatch order (reversed, and longest-first by a first launch's
    passes) and the frame queue (3 work-groups taking frame tickets for 7 frames) give the same
    bits as the default one-work-group-per-frame launch -- every frame is fitted on its own;
    with G = 2 the order maps (frame, part) tickets too.  A permutation of another length is
    SSF_E_ARG, and an out-of-range entry skips that frame (its output row is left as it was)."""
    import ssf
    fr = [frame(s, k, n_az=500) for s, k in ((1, 0), (2, 3), (3, 1), (4, 5), (5, 2), (6, 4), (7, 7))]
    F = len(fr)
    draws = np.random.default_rng(3).random((F, 3))
    fe = ssf.Frontend(64, device=dev.index)
    fe.mask_split(G)
    ref, bg_ref, _ = _run(fe, dev, [f[0] for f in fr], [f[1] for f in fr], draws=draws)
    assert np.all(ref[:, 16] == 0)
    longest = torch.from_numpy(np.argsort(-ref[:, 25], kind="stable").astype(np.int32)).to(dev)
    rev = torch.arange(F - 1, -1, -1, dtype=torch.int32, device=dev)
    for order, queue in ((rev, 0), (longest, 0), (None, 3), (longest, 3)):
        if G > 1 and queue:
            continue                         # the queue is the one-work-group-per-frame mode
        fe.mask_schedule(order, queue)
        out, bg, _ = _run(fe, dev, [f[0] for f in fr], [f[1] for f in fr], draws=draws)
        assert np.array_equal(out.view(np.uint64), ref.view(np.uint64)), (order, queue)
        assert np.array_equal(bg, bg_ref)
    fe.mask_schedule(rev[:F - 1])
    with pytest.raises(ssf.SSFError):
        _run(fe, dev, [f[0] for f in fr], [f[1] for f in fr], draws=draws)
    skip = torch.tensor([0, 1, 2, 3, 4, 5, 99], dtype=torch.int32, device=dev)   # frame 6 never runs
    fe.mask_schedule(skip)
    pts = torch.from_numpy(np.concatenate([f[0] for f in fr])).to(dev)
    fl = torch.from_numpy(np.concatenate([f[1] for f in fr])).to(dev)
    off, h_off = ssf.frame_offsets([f[0].shape[0] for f in fr], dev)
    out_buf = torch.full((F, 32), -7.0, dtype=torch.float64, device=dev)
    bg_buf = torch.empty(int(h_off[-1]), dtype=torch.uint8, device=dev)
    out, _ = fe.mask_pose(pts, fl, off, h_off, draws=draws, out=(out_buf, bg_buf))
    got = out.cpu().numpy()
    assert np.array_equal(got[:F - 1].view(np.uint64), ref[:F - 1].view(np.uint64))
    assert np.all(got[F - 1] == -7.0)
    fe.mask_schedule()


def test_frame_split_work_groups_take_several_tickets(oracle, dev):
    """Split G = 8 with n_frames * 8 > the resident work-groups (mask_pose_slots): the grid is
    capped at the slots, so work-groups take several (frame, part) tickets in order and reuse
    their LDS state across frames.  Every frame must equal the same frame fitted alone (one
    ticket per work-group: the per-part sums and their exchange order are the same), also with
    two such launches on two streams at once."""
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    fe.mask_split(8)
    props = torch.cuda.get_device_properties(dev)
    n_fr = props.multi_processor_count // 8 + 3          # 8 x n_fr > one work-group per CU
    batches = []
    for b in range(2):
        fr = [frame(40 + 50 * b + k, k % 3, n_az=60) for k in range(n_fr)]
        draws = np.array([[0.05 + 0.9 * ((k * 7 + b) % 11) / 11, 0.37, 0.81] for k in range(n_fr)])
        batches.append((fr, draws))
    # reference: every frame alone (8 work-groups, one ticket each)
    ref = []
    for fr, draws in batches:
        rows = []
        for k, f in enumerate(fr):
            o, bg, _ = _run(fe, dev, [f[0]], [f[1]], draws=draws[k:k + 1])
            rows.append((o[0][:26], bg))
        ref.append(rows)
    # one launch per batch, both batches on two streams at once
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    inputs = []
    for fr, draws in batches:
        pts = torch.from_numpy(np.concatenate([f[0] for f in fr])).to(dev)
        fl = torch.from_numpy(np.concatenate([f[1] for f in fr])).to(dev)
        off, h_off = ssf.frame_offsets([f[0].shape[0] for f in fr], dev)
        inputs.append((pts, fl, off, h_off, draws))
    torch.cuda.synchronize()
    outs = []
    for b, (pts, fl, off, h_off, draws) in enumerate(inputs):
        with torch.cuda.stream(streams[b]):
            o, bg = fe.mask_pose(pts, fl, off, h_off, draws=draws)
        outs.append((o, bg, h_off))
    torch.cuda.synchronize()
    for b, (o, bg, h_off) in enumerate(outs):
        o, bg = o.cpu().numpy(), bg.cpu().numpy()
        for k in range(n_fr):
            a, e = int(h_off[k]), int(h_off[k + 1])
            ro, rbg = ref[b][k]
            assert o[k, 16] == 0, (b, k, o[k, 16])
            assert np.array_equal(o[k, :26], ro), (b, k)
            assert np.array_equal(bg[a:e], rbg), (b, k)
    # and the fits are the reference's (sanity on a few frames)
    fr, draws = batches[0]
    o = outs[0][0].cpu().numpy()
    for k in (0, n_fr - 1):
        r = oracle.mask_and_pose(fr[k][0], fr[k][1], draws[k])
        assert int(o[k, 19]) == int(r["info"]["kmeans_iter"]) and int(o[k, 20]) == int(r["info"]["em_iter"])


def test_concurrent_streams_one_context(dev):
    """ssf_mask_pose_batch from one context on two streams back to back (the bench overlaps
    consecutive batches this way): every launch stages its draws in its own slot, so each result
    equals the same launch run alone."""
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    batches = []
    for k in range(3):
        fr = [frame(8 + k, 0, n_az=900), frame(9 + k, 1, n_az=900)]
        pts = torch.from_numpy(np.concatenate([f[0] for f in fr])).to(dev)
        fl = torch.from_numpy(np.concatenate([f[1] for f in fr])).to(dev)
        off, h_off = ssf.frame_offsets([f[0].shape[0] for f in fr], dev)
        draws = np.array([[0.1 + 0.2 * k, 0.3, 0.6], [0.9 - 0.1 * k, 0.5, 0.2]])
        batches.append((pts, fl, off, h_off, draws))
    ref = []
    for b in batches:
        o, bg = fe.mask_pose(b[0], b[1], b[2], b[3], draws=b[4])
        torch.cuda.synchronize()
        ref.append((o.cpu().numpy(), bg.cpu().numpy()))
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    outs = []
    for k, b in enumerate(batches):
        with torch.cuda.stream(streams[k % 2]):
            outs.append(fe.mask_pose(b[0], b[1], b[2], b[3], draws=b[4]))
    torch.cuda.synchronize()
    for (o, bg), (ro, rbg) in zip(outs, ref):
        assert np.array_equal(o.cpu().numpy()[:, :26], ro[:, :26])
        assert np.array_equal(bg.cpu().numpy(), rbg)


def test_gt_and_given_masks(oracle, dev):
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    p, fl, fg = frame(7, 2)
    out, bg, _ = _run(fe, dev, [p], [fl], mode="gt", mask=[fg])
    rc, R, t = oracle.kabsch(p.astype(np.float64) + fl, p.astype(np.float64), (fg == 0).astype(np.uint8))
    assert out[0, 16] == 0 and rc == 0
    assert np.array_equal(bg, (fg == 0).astype(np.uint8))
    assert np.abs(out[0, 0:3] - t).max() < 1e-6 and np.abs(out[0, 7:16].reshape(3, 3) - R).max() < 1e-9
    out2, bg2, _ = _run(fe, dev, [p], [fl], mode="given", mask=[(fg == 0).astype(np.uint8)])
    assert np.abs(out2[0, :16] - out[0, :16]).max() == 0.0


def test_reflection_status(dev):
    """det(R) < 0: the reference raises TypeError (`Vt.T & U.T`, PointCloudOdometry_noSeg.py:33);
    here status SSF_POSE_REFLECTION, or the fixed rotation with reflection=1."""
    import ssf
    g = np.load(os.path.join(GOLDEN, "kabsch_ref.npz"))
    assert int(g["refl_raises_typeerror"]) == 1
    src, dst = g["refl_src"], g["refl_dst"]
    fe = ssf.Frontend(64, device=dev.index)
    ones = [np.ones(len(dst), np.uint8)]
    out, _, _ = _run(fe, dev, [dst], [src - dst], mode="given", mask=ones)
    assert out[0, 16] == -2
    out, _, _ = _run(fe, dev, [dst], [src - dst], mode="given", mask=ones, reflection=1)
    R = out[0, 7:16].reshape(3, 3)
    assert abs(np.linalg.det(R) - 1.0) < 1e-9


def test_mask_and_pose_per_frame_status(dev):
    """errors='status': a batch with one failing frame (empty background: every point masked out)
    keeps the other frames' poses and reports each frame's status; the default raises."""
    import ssf
    p, fl, fg = frame(7, 2)
    bgm = (fg == 0).astype(np.uint8)
    pts = np.concatenate([p, p]); flow = np.concatenate([fl, fl])
    gm = np.concatenate([fg, np.ones_like(fg)])                    # frame 1: all foreground
    r = ssf.mask_and_pose(pts, flow, mode="gt", gt_mask=gm, frame_sizes=[len(p), len(p)],
                          device=dev.index, errors="status")
    st = r["info"]["status"]
    assert st[0] == 0 and st[1] == ssf._abi.POSE_EMPTY, st
    one = ssf.mask_and_pose(p, fl, mode="gt", gt_mask=fg, device=dev.index)
    assert np.array_equal(r[0][0], one[0]) and np.array_equal(r[1][0], one[1])
    with pytest.raises(ValueError):
        ssf.mask_and_pose(pts, flow, mode="gt", gt_mask=gm, frame_sizes=[len(p), len(p)], device=dev.index)
    with pytest.raises(ValueError):
        ssf.mask_and_pose(p, fl, mode="gt", gt_mask=fg, device=dev.index, errors="ignore")
    assert bgm.sum() > 0


def _rot_angle(Ra, Rb):
    """Rotation angle of Ra^T Rb, from ||Ra - Rb||_F = 2 sqrt(2) sin(theta / 2) (no arccos near 1)."""
    return float(2.0 * np.arcsin(min(1.0, np.linalg.norm(Ra - Rb) / (2.0 * np.sqrt(2.0)))))


def test_kabsch_golden(dev):
    """slove_RT_by_SVD golden cases: float64 inputs through the f64-storage kernel
    (ssf_mask_pose_batch_f64) against the f64 reference -- north_star bars 1e-5 m / 1e-6 rad."""
    import ssf
    g = np.load(os.path.join(GOLDEN, "kabsch_ref.npz"))
    fe = ssf.Frontend(64, device=dev.index)
    for c in range(4):
        src, dst = g[f"src{c}"], g[f"dst{c}"]
        assert src.dtype == np.float64
        pts = torch.from_numpy(np.ascontiguousarray(dst)).to(dev)
        fl = torch.from_numpy(np.ascontiguousarray(src - dst)).to(dev)
        off, h_off = ssf.frame_offsets([len(dst)], dev)
        ones = torch.ones(len(dst), dtype=torch.uint8, device=dev)
        out, _ = fe.mask_pose(pts, fl, off, h_off, mode="given", mask_in=ones)
        o = out[0].cpu().numpy()
        assert o[16] == 0
        R = o[7:16].reshape(3, 3)
        assert _rot_angle(R, g[f"R{c}"]) < 1e-6, c
        assert np.abs(o[0:3] - g[f"t{c}"]).max() < 1e-5, c
        assert np.abs(R - g[f"R{c}"]).max() < 1e-9, c          # observed ~1e-15


def test_kabsch_golden_f32_inputs(dev):
    """The float32 LiDAR path on the same cases: inputs rounded to f32 (|x| ~ 10-40 m, so the
    rounding itself moves t by up to ~1e-5 m): R within 1e-5, t within 1e-4."""
    import ssf
    g = np.load(os.path.join(GOLDEN, "kabsch_ref.npz"))
    fe = ssf.Frontend(64, device=dev.index)
    for c in range(4):
        src = g[f"src{c}"].astype(np.float32)
        dst = g[f"dst{c}"].astype(np.float32)
        out, _, _ = _run(fe, dev, [dst], [src - dst], mode="given", mask=[np.ones(len(dst), np.uint8)])
        assert out[0, 16] == 0
        assert np.abs(out[0, 7:16].reshape(3, 3) - g[f"R{c}"]).max() < 1e-5
        assert np.abs(out[0, 0:3] - g[f"t{c}"]).max() < 1e-4


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "gmm_noseg_case*.npz"))))
def test_gmm_f64_storage_matches_golden(dev, path):
    """The f64-storage kernel on the golden frames given as float64 (the reference's own
    `points = pos1.astype(float64)`): same labels, k-means++ indices, iteration counts and pose."""
    import ssf
    g = np.load(path)
    fe = ssf.Frontend(64, device=dev.index)
    pts = torch.from_numpy(g["pos1"].astype(np.float64)).to(dev)
    fl = torch.from_numpy(g["flow"].astype(np.float64)).to(dev)
    off, h_off = ssf.frame_offsets([len(g["pos1"])], dev)
    out, bg = fe.mask_pose(pts, fl, off, h_off, mode="gmm", draws=g["draws"][None, :])
    o = out[0].cpu().numpy()
    assert o[16] == 0
    assert [int(o[22]), int(o[23])] == [int(v) for v in g["kmeans_pp_idx"]]
    assert int(o[19]) == int(g["kmeans_n_iter"]) and int(o[20]) == int(g["gmm_n_iter"])
    bg_ref = (g["labels"] == int(g["bg_label"])).astype(np.uint8)
    assert np.array_equal(bg.cpu().numpy(), bg_ref)
    assert abs(o[24] - float(g["gmm_lower_bound"])) < 1e-9
    assert _rot_angle(o[7:16].reshape(3, 3), g["R"]) < 1e-6
    assert np.abs(o[0:3] - g["t"]).max() < 1e-5


def test_reference_named_python_api(dev):
    """ssf.slove_RT_by_SVD / ssf.mask_and_pose keep the reference signatures and errors"""
    import ssf
    g = np.load(os.path.join(GOLDEN, "kabsch_ref.npz"))
    R, t = ssf.slove_RT_by_SVD(g["src2"], g["dst2"])          # float64 in: no input rounding
    assert R.shape == (3, 3) and t.shape == (3, 1)
    assert _rot_angle(R, g["R2"]) < 1e-6 and np.abs(t.ravel() - g["t2"]).max() < 1e-5
    with pytest.raises(ValueError):
        ssf.slove_RT_by_SVD(g["refl_src"], g["refl_dst"])
    R2, _ = ssf.slove_RT_by_SVD(g["refl_src"], g["refl_dst"], reflection="fix")
    assert abs(np.linalg.det(R2) - 1) < 1e-9
    c = np.load(os.path.join(GOLDEN, "gmm_noseg_case0.npz"))
    res = ssf.mask_and_pose(c["pos1"], c["flow"], seed=int(c["seed"]))
    assert np.abs(res["para_t_q"][0] - c["para_t_q"]).max() < 1e-6
    R1, t1, q1, bg1 = res                                       # the SURVEY §8(b) tuple
    assert R1.shape == (3, 3) and t1.shape == (3, 1) and q1.shape == (4,)
    assert _rot_angle(R1, c["R"]) < 1e-6 and np.abs(t1.ravel() - c["t"]).max() < 1e-5
    assert bg1 is res["bg_mask"] and res.info["em_iter"][0] == int(c["gmm_n_iter"])
    bg_ref = (c["labels"] == int(c["bg_label"])).astype(np.uint8)
    assert np.array_equal(res["bg_mask"].cpu().numpy(), bg_ref)
    gt = ssf.mask_and_pose(c["pos1"], c["flow"], mode="gt", gt_mask=c["s_fg_mask"])
    assert gt["bg_mask"].cpu().numpy().sum() == int((c["s_fg_mask"] == 0).sum())


@pytest.mark.parametrize("case", range(4))
def test_asf_f32_block(oracle, dev, case):
    """ASF block on float32 network output (main_sju_occ_ros.py:256-284): the f32-storage kernel
    (f64 arithmetic) equals the oracle, and stays within the documented deviation bars of the
    reference's own float32 run (tests/test_oracle_golden.py ASF_BARS)."""
    from test_oracle_golden import ASF_BARS
    import ssf
    g = np.load(os.path.join(GOLDEN, "gmm_asf_f32.npz"))
    p, f, d = g[f"pos1_{case}"], g[f"flow_{case}"], g[f"draws_{case}"]
    res = ssf.mask_and_pose(p, f, draws=d[None, :])
    ref = oracle.mask_and_pose(p, f, d)
    bg = res["bg_mask"].cpu().numpy()
    assert (bg == ref["bg_mask"]).mean() >= 0.999
    assert np.abs(res["t"][0] - ref["t"]).max() < 1e-5 and _rot_angle(res["R"][0], ref["R"]) < 1e-6
    bg_ref = (g[f"labels_{case}"] == int(g[f"bg_label_{case}"])).astype(np.uint8)
    assert (bg == bg_ref).mean() >= ASF_BARS["agree"]
    assert np.abs(res["R"][0] - g[f"R_{case}"]).max() < ASF_BARS["R"]
    assert np.abs(res["t"][0] - g[f"t_{case}"]).max() < ASF_BARS["t"]
    # per frame against the float32 reference's own sensitivity (a19, make_asf_sensitivity.py):
    # stable frames -> identical mask and EM iteration count, pose = the exact Kabsch of that mask
    from test_oracle_golden import asf_check
    asf_check(case, bg, res["info"]["em_iter"][0], res["t"][0])


@pytest.mark.parametrize("case", range(4))
def test_asf_f32_kabsch_tail(oracle, dev, case):
    """a19 closed: the GMM on device + ssf_kabsch_f32_batch, the float32
    slove_RT_by_SVD / Quaternion tail of main_sju_occ_ros.py:273-284.  Against the oracle's
    float32 restatement (orc_kabsch_f32) on the same inputs, and on the stable frames against the
    reference's own float32 R / t within 1e-6 (tests/test_oracle_golden.py F32_TAIL_BAR)."""
    import ssf
    from test_oracle_golden import F32_TAIL_BAR, asf_case_bars
    g = np.load(os.path.join(GOLDEN, "gmm_asf_f32.npz"))
    p, f, d = g[f"pos1_{case}"], g[f"flow_{case}"], g[f"draws_{case}"]
    res = ssf.mask_and_pose(p, f, draws=d[None, :], kabsch_dtype="float32")
    ref = oracle.mask_and_pose(p, f, d, kabsch_dtype="float32")
    bg = res["bg_mask"].cpu().numpy()
    assert ref["rc"] == 0
    if np.array_equal(bg, ref["bg_mask"]):          # same rows: the same float32 arithmetic
        assert np.abs(res["R"][0] - ref["R"]).max() < 1e-6
        assert np.abs(res["t"][0] - ref["t"]).max() < 1e-6
        assert np.abs(res["q_xyzw"][0] - ref["q_xyzw"]).max() < 1e-6
    assert np.array_equal(res["R"][0], res["R"][0].astype(np.float32))   # float32 values
    b = asf_case_bars(case)
    bg_ref = (g[f"labels_{case}"] == int(g[f"bg_label_{case}"])).astype(np.uint8)
    if b["stable"]:
        assert np.array_equal(bg, bg_ref)
        assert int(res["info"]["em_iter"][0]) == b["n_iter"]
        assert np.abs(res["R"][0] - g[f"R_{case}"]).max() < F32_TAIL_BAR["R"]
        assert np.abs(res["t"][0] - g[f"t_{case}"]).max() < F32_TAIL_BAR["t"]
    else:
        assert np.abs(res["t"][0] - g[f"t_{case}"]).max() <= b["t_spread"]
    # the fit fields of the mask kernel are kept
    assert int(res["info"]["em_iter"][0]) >= 1 and res["info"]["n_bg"][0] == bg.sum()


def test_slove_RT_by_SVD_float32(oracle, dev):
    """slove_RT_by_SVD(src, dst, kabsch_dtype='float32') on float32 arrays = numpy's own float32
    run of the reference function's lines (:455-473), ValueError on a reflection, on no rows."""
    import ssf
    rng = np.random.default_rng(11)
    dst = (rng.standard_normal((6000, 3)) * 20).astype(np.float32)
    ang = 0.03
    Rt = np.array([[np.cos(ang), -np.sin(ang), 0], [np.sin(ang), np.cos(ang), 0], [0, 0, 1]])
    src = (dst @ Rt.T + np.array([0.8, -0.1, 0.02]) + rng.standard_normal((6000, 3)) * 0.01).astype(np.float32)
    R, t = ssf.slove_RT_by_SVD(src, dst, kabsch_dtype="float32")
    sm, dm = src.mean(axis=0, keepdims=True), dst.mean(axis=0, keepdims=True)
    U, S, Vt = np.linalg.svd((src - sm).T @ (dst - dm))
    Rn = Vt.T @ U.T
    tn = -Rn @ sm.T + dm.T
    assert R.shape == (3, 3) and t.shape == (3, 1)
    assert np.abs(R - Rn).max() < 1e-6 and np.abs(t - tn).max() < 2e-6
    with pytest.raises(ValueError):
        ssf.slove_RT_by_SVD(src, -src, kabsch_dtype="float32")
    R2, _ = ssf.slove_RT_by_SVD(src, -src, reflection="fix", kabsch_dtype="float32")
    assert abs(np.linalg.det(R2) - 1) < 1e-5
    c = np.load(os.path.join(GOLDEN, "gmm_noseg_case0.npz"))
    with pytest.raises(ValueError):
        ssf.mask_and_pose(c["pos1"], c["flow"], mode="given", gt_mask=np.zeros(len(c["pos1"]), np.uint8),
                          kabsch_dtype="float32")


def test_frame_above_32bit_offsets_rejected(dev):
    """The streaming loops address a frame with 32-bit byte offsets (mask_pose.hip load3_off):
    ssf_mask_pose_batch rejects a frame above 2^32 / 12 points (f32) or 2^32 / 24 (f64) with
    SSF_E_ARG before anything is launched (the device pointers are never dereferenced here)."""
    import ctypes as C
    import ssf
    from ssf import _abi
    from ssf.frontend import MASK_MODES, _stream
    MASK_GMM = MASK_MODES["gmm"]
    fe = ssf.Frontend(64, device=dev.index)
    lib = _abi.lib()
    fake = C.c_void_p(16)                               # never touched: the check comes first
    for name, bytes_per_point in (("ssf_mask_pose_batch", 12), ("ssf_mask_pose_batch_f64", 24)):
        n = (2 ** 32 - 1) // bytes_per_point + 1
        h_off = np.array([0, n], dtype=np.int64)
        rc = getattr(lib, name)(fe._h, _stream(fe.device), 1, fake, fake, fake,
                                C.c_void_p(h_off.ctypes.data), MASK_GMM, None, None, 0, None, fake)
        assert rc == _abi.SSF_E_ARG, (name, n, rc)
