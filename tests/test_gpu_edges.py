"""Edge features + point-to-line residuals (beyond the reference, off unless called) on the GPU
vs the CPU restatement oracle/edge_oracle.c.  Parity with the reference is unpinned (it has no
edge path); the bars are those of the planar path: feature lists and line tables bit-exact,
per-step poses within 1e-5 m / 1e-6 rad."""
import numpy as np
import pytest
import torch

from helpers import frame

pytestmark = pytest.mark.gpu
TOL_T, TOL_R = 1e-5, 1e-6


def _angle(q1, q2):
    d = abs(float(np.dot(q1 / np.linalg.norm(q1), q2 / np.linalg.norm(q2))))
    return 2.0 * np.arcsin(min(1.0, np.sqrt(max(0.0, 1.0 - d * d))))


def _features(fe, dev, clouds):
    import ssf
    pts = torch.from_numpy(np.concatenate(clouds)).to(dev)
    off, h_off = ssf.frame_offsets([c.shape[0] for c in clouds], dev)
    return pts, off, h_off, fe.extract_features_batch(pts, off, h_off)


def _pair(b, a, c):
    import ssf
    last = ssf.PlaneBatch(b.xyzi, b.count[a:a + 1], b.off[a:a + 2], b.h_off[a:a + 2], b.max_points)
    curr = ssf.PlaneBatch(b.xyzi, b.count[c:c + 1], b.off[c:c + 2], b.h_off[c:c + 2], b.max_points)
    return last, curr


@pytest.mark.parametrize("rows,n_az", [(64, 1875), (16, 1800), (16, 4500)])
def test_edge_features_bitexact(oracle, dev, rows, n_az):
    import ssf
    fe = ssf.Frontend(rows, device=dev.index)
    fe.edge_config()
    clouds = [frame(3, k, n_rows=rows, n_az=n_az)[0] for k in range(3)]
    pts, off, h_off, (pb, eb) = _features(fe, dev, clouds)
    pb_ref = fe.extract_planes_batch(pts, off, h_off)          # the planes are untouched by edges
    torch.cuda.synchronize()
    for f, c in enumerate(clouds):
        P, E = oracle.extract_features(c, rows)
        assert np.array_equal(pb.frame(f).cpu().numpy(), P), f
        assert np.array_equal(pb_ref.frame(f).cpu().numpy(), P), f
        g = eb.frame(f).cpu().numpy()
        assert len(E) > 50 and np.array_equal(g.view(np.uint32), E.view(np.uint32)), (f, len(g), len(E))


def test_edge_config_and_masked(oracle, dev):
    """custom edge_min / edge_span, and the keep mask (edges of the kept points only)"""
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    fe.edge_config(edge_min=0.2, edge_span=5)
    c = frame(4, 0, n_az=1875)[0]
    keep = (np.arange(len(c)) % 7 != 3).astype(np.uint8)
    pts = torch.from_numpy(c).to(dev)
    off, h_off = ssf.frame_offsets([len(c)], dev)
    pb, eb = fe.extract_features_batch(pts, off, h_off, keep=torch.from_numpy(keep).to(dev))
    torch.cuda.synchronize()
    P, E = oracle.extract_features(c[keep != 0], 64, edge_min=0.2, edge_span=5)
    assert np.array_equal(pb.frame(0).cpu().numpy(), P)
    assert np.array_equal(eb.frame(0).cpu().numpy(), E)


def test_edge_table_bitexact(oracle, dev):
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    clouds = [frame(5, k, n_az=1875)[0] for k in range(2)]
    _, _, _, (pb, eb) = _features(fe, dev, clouds)
    line, valid = fe.edge_table(eb)
    torch.cuda.synchronize()
    for f in range(2):
        E = eb.frame(f).cpu().numpy()
        L, V = oracle.edge_table(E)
        o, m = int(eb.h_off[f]), len(E)
        assert np.array_equal(valid[o:o + m].cpu().numpy(), V.astype(np.uint8)), f
        assert 0.3 < V.mean() < 0.95
        assert np.array_equal(line[o:o + m].cpu().numpy().view(np.uint32), L.view(np.uint32)), f


@pytest.mark.parametrize("solver,mode,iters", [("gn", 1, 10), ("ceres_lm", 0, 8)])
def test_register_with_edges_per_step(oracle, dev, solver, mode, iters):
    import ssf
    fe = ssf.Frontend(64, device=dev.index, solver=solver, max_iter=iters)
    clouds = [frame(6, k, n_az=1875)[0] for k in range(2)]
    _, _, _, (pb, eb) = _features(fe, dev, clouds)
    table = fe.plane_table(pb)
    etable = fe.edge_table(eb)
    last, curr = _pair(pb, 0, 1)
    last_e, curr_e = _pair(eb, 0, 1)
    q0 = np.array([0.0, 0.0, 0.001, 1.0]); q0 /= np.linalg.norm(q0)
    t0 = np.array([0.9, 0.01, 0.0])
    pose = torch.tensor([[*q0, *t0]], dtype=torch.float64, device=dev)
    res = fe.register(last, table, curr, pose, want_log=True, edges=(last_e, etable, curr_e))
    torch.cuda.synchronize()
    P0, P1 = pb.frame(0).cpu().numpy(), pb.frame(1).cpu().numpy()
    E0, E1 = eb.frame(0).cpu().numpy(), eb.frame(1).cpu().numpy()
    q, t, log, c, ce = oracle.register_pair_edges(P0, P1, E0, E1, 0.05, mode=mode, max_iter=iters,
                                                  q_init=q0, t_init=t0)
    assert int(res["ncorr"][0]) == c and int(res["ncorr_edge"][0]) == ce and ce > 50
    nl = int(res["nlog"][0])
    assert nl == log.shape[0]
    glog = res["log"][0, :nl].cpu().numpy()
    for i in range(nl):
        assert glog[i, 8] == log[i, 8], i
        assert np.abs(glog[i, 4:7] - log[i, 4:7]).max() < TOL_T, i
        assert _angle(glog[i, :4], log[i, :4]) < TOL_R, i
    got = res["pose_rel"][0].cpu().numpy()
    assert np.abs(got[4:] - t).max() < TOL_T and _angle(got[:4], q) < TOL_R


def test_register_edges_empty_equals_planes(oracle, dev):
    """edge_min above every curvature: no edge block, the same pose as ssf_register_batch"""
    import ssf
    fe = ssf.Frontend(64, device=dev.index, solver="gn", max_iter=10)
    fe.edge_config(edge_min=1e30)
    clouds = [frame(7, k, n_az=1875)[0] for k in range(2)]
    _, _, _, (pb, eb) = _features(fe, dev, clouds)
    assert int(eb.count.sum()) == 0
    table = fe.plane_table(pb)
    etable = fe.edge_table(eb)
    last, curr = _pair(pb, 0, 1)
    last_e, curr_e = _pair(eb, 0, 1)
    p1 = ssf.identity_poses(1, dev)
    p2 = ssf.identity_poses(1, dev)
    r1 = fe.register(last, table, curr, p1, edges=(last_e, etable, curr_e))
    r2 = fe.register(last, table, curr, p2)
    torch.cuda.synchronize()
    assert int(r1["ncorr_edge"][0]) == 0 and int(r1["ncorr"][0]) == int(r2["ncorr"][0])
    assert torch.equal(p1, p2)
