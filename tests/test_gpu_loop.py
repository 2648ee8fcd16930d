"""Loop-closure registration (src/mapOptmization.cpp:200-272) on the GPU
vs the CPU oracle (oracle/loop_oracle.c, PCL 1.10 VoxelGrid / IterativeClosestPoint
restated; parity against PCL itself is unpinned).

Bars: voxel grid bit-exact (same voxel keys, same in-order float centroid sums); ICP final
transform within 1e-5 (rotation) / 1e-4 m, identical iteration count and convergence state,
fitness within 1e-6 relative (the GPU sums its double reductions in a different order).
"""
import numpy as np
import pytest
import torch

from helpers import frame

pytestmark = pytest.mark.gpu


def _planes(O, seq, k):
    pts, _, _ = frame(seq, k)
    return O.extract_planes(pts, 64)


def _dev_cat(clouds, dev):
    import ssf
    x = torch.from_numpy(np.concatenate(clouds).astype(np.float32)).to(dev) if clouds else \
        torch.zeros(0, 4, device=dev)
    off, h_off = ssf.frame_offsets([c.shape[0] for c in clouds], dev)
    return x, off, h_off


def test_voxel_grid_batch_bitexact(oracle, dev):
    from ssf import Frontend, loop
    O = oracle
    rng = np.random.default_rng(3)
    clouds = [_planes(O, 0, 0), np.zeros((0, 4), np.float32), _planes(O, 1, 2),
              np.concatenate([rng.uniform(-3, 3, (5000, 3)), rng.uniform(0, 64, (5000, 1))], 1).astype(np.float32)]
    # duplicated points (several per voxel) and a cloud sitting on voxel boundaries
    clouds.append(np.repeat(clouds[0][:500], 3, axis=0))
    g = np.stack(np.meshgrid(np.arange(20), np.arange(20), np.arange(3), indexing="ij"), -1).reshape(-1, 3) * 0.1
    clouds.append(np.concatenate([g, np.ones((g.shape[0], 1))], 1).astype(np.float32))
    fe = Frontend(64, device=dev.index or 0)
    x, off, h_off = _dev_cat(clouds, dev)
    for leaf in (0.1, 0.4):
        out, cnt = loop.voxel_grid(fe, x, off, h_off, leaf)
        torch.cuda.synchronize()
        cnt = cnt.cpu().numpy()
        for c, cl in enumerate(clouds):
            ref = O.voxel_grid(cl, leaf) if cl.shape[0] else np.zeros((0, 4), np.float32)
            o = int(h_off[c])
            got = out[o:o + int(cnt[c])].cpu().numpy()
            assert got.shape == ref.shape, (leaf, c, got.shape, ref.shape)
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (leaf, c)


def test_voxel_grid_leaf_too_small_passes_through(oracle, dev):
    """PCL's overflow guard (dx*dy*dz > INT32_MAX): the input is returned unchanged."""
    from ssf import Frontend, loop
    cl = np.array([[0, 0, 0, 1], [1000, 1000, 1000, 2], [3, 4, 5, 3]], np.float32)
    fe = Frontend(64, device=dev.index or 0)
    got = loop.voxel_grid_one(fe, torch.from_numpy(cl).to(dev), 0.01).cpu().numpy()
    ref = oracle.voxel_grid(cl, 0.01)
    assert np.array_equal(got, cl) and np.array_equal(ref, cl)


def _check_icp(got, ref):
    assert got["state"] == ref["state"], (got["state"], ref["state"])
    assert got["iterations"] == ref["iterations"], (got["iterations"], ref["iterations"])
    assert got["converged"] == ref["converged"]
    assert np.abs(got["T"][:3, :3] - ref["T"][:3, :3]).max() < 1e-5, (got["T"], ref["T"])
    assert np.abs(got["T"][:3, 3] - ref["T"][:3, 3]).max() < 1e-4, (got["T"], ref["T"])
    assert abs(got["fitness"] - ref["fitness"]) <= 1e-6 * max(1.0, abs(ref["fitness"]))


def test_icp_consecutive_frames_vs_oracle(oracle, dev):
    """Plane clouds of consecutive synthetic frames (~1 m motion): the loop-closure ICP
    parameters of mapOptmization.cpp:225-229."""
    from ssf import Frontend, loop
    O = oracle
    src, tgt = _planes(O, 0, 1), _planes(O, 0, 0)
    fe = Frontend(64, device=dev.index or 0)
    got = loop.icp(fe, torch.from_numpy(src).to(dev), torch.from_numpy(tgt).to(dev))
    ref = O.icp(src, tgt)
    _check_icp(got, ref)
    assert ref["converged"] and ref["fitness"] < 2.0   # different samplings of the same scene


def test_icp_batch_guess_and_degenerate(oracle, dev):
    """Batched problems with guesses, a known rigid motion, and a problem with < 3
    correspondences inside a tiny gate (NO_CORRESPONDENCES, not converged)."""
    from ssf import Frontend, loop
    O = oracle
    a, b = _planes(O, 1, 0), _planes(O, 1, 1)
    ang = 0.03
    R = np.array([[np.cos(ang), -np.sin(ang), 0], [np.sin(ang), np.cos(ang), 0], [0, 0, 1]])
    moved = a.copy()
    moved[:, :3] = (a[:, :3].astype(np.float64) @ R.T + [0.4, -0.3, 0.05]).astype(np.float32)
    guess = np.eye(4, dtype=np.float32)
    guess[:3, 3] = [0.3, -0.2, 0.0]
    probs = [(b, a, np.eye(4, dtype=np.float32)), (a, moved, guess), (a[:200], moved[:200] + 100.0, np.eye(4, dtype=np.float32))]
    fe = Frontend(64, device=dev.index or 0)
    s, so, hso = _dev_cat([p[0] for p in probs], dev)
    t, to, hto = _dev_cat([p[1] for p in probs], dev)
    params = loop.icp_params(max_corr_dist=50.0)
    got = loop.icp_batch(fe, s, so, hso, t, to, hto, params, np.stack([p[2] for p in probs]))
    for k, (sk, tk, gk) in enumerate(probs):
        mc = 50.0
        ref = O.icp(sk, tk, max_corr_dist=mc, guess=gk)
        _check_icp(got[k], ref)
    assert got[2]["state"] == "no_correspondences" and not got[2]["converged"]
    assert got[1]["converged"]
    Rt = got[1]["T"]
    assert np.abs(Rt[:3, :3] - R).max() < 1e-3 and np.abs(Rt[:3, 3] - [0.4, -0.3, 0.05]).max() < 1e-2


def test_loop_closer_detects_revisit(dev):
    """A sequence that returns to its start after > 20 s: the keyframe logic (isKeyFrame,
    detectLoopFrameID, getLoopLocalMap) fires, the local map / ICP run on the GPU, and the
    correction removes a deliberate 0.5 m odometry drift on the revisit."""
    from ssf import Frontend, loop, synth
    from oracle import oracle as O
    fe = Frontend(64, device=dev.index or 0)
    sc = synth.Scene(0)
    lc = loop.LoopCloser(fe)
    R0, p0 = synth.ego_pose(0, 0)
    T0 = np.eye(4); T0[:3, :3] = R0.numpy(); T0[:3, 3] = p0.numpy()
    # 30 frames forward (every second one becomes a keyframe: a 1 m arc is a chord below 1 m),
    # then a revisit of frames 0..5, so the loop keys are > 10 keyframes apart (getLoopLocalMap
    # takes the 10 keyframes either side of the loop candidate)
    seq = list(range(30)) + list(range(6))
    n_fwd = None
    cons = []
    for i, k in enumerate(seq):
        f = synth.scan(0, k, n_az=600, scene=sc)
        pl = torch.from_numpy(O.extract_planes(f["pos1"].numpy(), 64)).to(dev)
        R, p = synth.ego_pose(0, k)
        Tk = np.eye(4); Tk[:3, :3] = R.numpy(); Tk[:3, 3] = p.numpy()
        T = np.linalg.inv(T0) @ Tk                  # odometry relative to the first frame
        revisit = i >= 30
        if revisit and n_fwd is None:
            n_fwd = len(lc.key6d)
        if revisit:
            T[0, 3] += 0.5                          # drift
        yaw = np.arctan2(T[1, 0], T[0, 0])
        q = (0.0, 0.0, np.sin(yaw / 2), np.cos(yaw / 2))
        _, c, _ = lc.process(pl, q, T[:3, 3], 0.1 * i + (30.0 if revisit else 0.0))
        if c is not None:
            cons.append(c)
    assert cons, "no loop constraint"
    c = cons[0]
    assert c.key_pre < n_fwd <= c.key_cur and c.key_cur - c.key_pre > 10, (c.key_pre, c.key_cur, n_fwd)
    assert abs(c.correction[0, 3] + 0.5) < 0.1, c.correction
    assert abs(c.correction[1, 3]) < 0.1 and c.noise < 0.2
