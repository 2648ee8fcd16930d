"""Edge features + point-to-line residuals (beyond the reference; oracle/edge_oracle.c) -- CPU
known-answer tests of the restatement the GPU kernels are checked against.  Parity with the
reference is unpinned by construction (the reference is planar / point-to-plane only)."""
import numpy as np
import pytest

from helpers import frame


def _rot(ax, ang):
    ax = np.asarray(ax, float) / np.linalg.norm(ax)
    K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


def test_sym3_eig_known(oracle):
    w, V = oracle.sym3_eig(np.diag([3.0, 1.0, 2.0]))
    assert np.allclose(sorted(w), [1, 2, 3]) and np.allclose(np.abs(V), np.eye(3))
    R = _rot([1, 2, 3], 0.7)
    A = R @ np.diag([5.0, 2.0, 0.5]) @ R.T
    w, V = oracle.sym3_eig(A)
    order = np.argsort(-w)
    assert np.allclose(w[order], [5, 2, 0.5], atol=1e-12)
    for k, col in enumerate(order):
        assert abs(abs(V[:, col] @ R[:, k]) - 1) < 1e-12


def test_select_edges_greedy_spacing(oracle):
    # one ring in the 64 profile's middle row: a straight wall with a sharp corner at index 40
    n = 80
    x = np.concatenate([np.linspace(0, 4, 41), np.full(39, 4.0)])
    y = np.concatenate([np.full(41, 10.0), np.linspace(10, 14, 40)[1:]])
    rx = np.stack([x, y, np.zeros(n), np.arange(n) + 0.30], 1).astype(np.float32)
    off = np.zeros(65, np.int64)
    off[31:] = n                                  # every point in row 30
    cv = oracle.curvature(rx, off, 64)
    assert cv[:30].max() < 1e-6 and cv[50:].max() < 1e-6 and cv[40] > 1.0
    # the first point (in row order) whose 11-tap window reaches the corner is selected, and the
    # spacing rule then skips the rest of the corner
    e = oracle.select_edges(rx, cv, off, 64, edge_min=0.5, edge_span=10)
    first = int(np.argmax(cv > 0.5))
    assert len(e) == 1 and int(round(float(e[0][3]) - 0.30)) == first and 35 <= first <= 40
    e2 = oracle.select_edges(rx, cv, off, 64, edge_min=0.01, edge_span=3)
    idx = [int(round(float(p[3]) - 0.30)) for p in e2]   # index in row
    assert len(idx) >= 3 and all(b - a >= 3 for a, b in zip(idx, idx[1:]))
    assert all(35 <= i <= 45 for i in idx)


def test_edge_table_line_and_blob(oracle):
    d = np.array([1.0, 2.0, 0.5]) / np.linalg.norm([1.0, 2.0, 0.5])
    line = np.array([1.0, 1.0, 1.0]) + np.outer(np.arange(10) * 0.1, d)
    # a regular pentagon: every point's 5-NN is the whole pentagon, isotropic in its plane
    ang = 2 * np.pi * np.arange(5) / 5
    blob = np.array([20.0, 0.0, 0.0]) + 0.3 * np.stack([np.cos(ang), np.sin(ang), np.zeros(5)], 1)
    far = np.array([[40.0, 0, 0], [41.5, 0, 0], [43.0, 0, 0], [44.5, 0, 0], [46.0, 0, 0]])   # gate: 5th NN > 1 m
    pts = np.zeros((20, 4), np.float32)
    pts[:10, :3], pts[10:15, :3], pts[15:, :3] = line, blob, far
    L, valid = oracle.edge_table(pts)
    assert valid[:10].all() and not valid[10:].any()
    for a in range(10):
        u = L[a, 3:]
        assert abs(abs(float(u @ d)) - 1) < 1e-5 and u[np.argmax(np.abs(u))] > 0
        # the centroid of the 5 nearest line points lies on the line
        c = L[a, :3] - np.array([1.0, 1.0, 1.0])
        assert np.linalg.norm(c - (c @ d) * d) < 1e-5


def test_point_to_line_recovers_known_motion(oracle):
    """planes + edges of one synthetic scan and of the same scan moved by a known (q, t): the
    LM solution with the point-to-line blocks recovers the motion."""
    pts = frame(2, 0, n_az=1875)[0]
    R = _rot([0.1, 0.2, 1.0], 0.01)
    t = np.array([0.30, -0.05, 0.02])
    moved = ((pts - t) @ R).astype(np.float32)       # curr = R^T (last - t): last = R curr + t
    P0, E0 = oracle.extract_features(pts, 64)
    P1, E1 = oracle.extract_features(moved, 64)
    assert len(E0) > 100 and len(E1) > 100
    q, tt, log, c, ce = oracle.register_pair_edges(P0, P1, E0, E1, 0.05, mode=oracle.MODE_CERES_LM,
                                                   max_iter=8)
    assert c > 100 and ce > 20 and len(log) > 0
    w = q[3]
    Rq = np.array([[1 - 2 * (q[1] ** 2 + q[2] ** 2), 2 * (q[0] * q[1] - q[2] * w), 2 * (q[0] * q[2] + q[1] * w)],
                   [2 * (q[0] * q[1] + q[2] * w), 1 - 2 * (q[0] ** 2 + q[2] ** 2), 2 * (q[1] * q[2] - q[0] * w)],
                   [2 * (q[0] * q[2] - q[1] * w), 2 * (q[1] * q[2] + q[0] * w), 1 - 2 * (q[0] ** 2 + q[1] ** 2)]])
    assert np.abs(Rq - R).max() < 2e-3 and np.abs(tt - t).max() < 2e-2


def test_edges_off_equals_planes_only(oracle):
    """No edge blocks (empty edge clouds) -> exactly the planar registration."""
    P0 = oracle.extract_planes(frame(1, 0, n_az=1200)[0], 64)
    P1 = oracle.extract_planes(frame(1, 1, n_az=1200)[0], 64)
    e = np.zeros((0, 4), np.float32)
    q, t, log, c, ce = oracle.register_pair_edges(P0, P1, e, e, 0.05, mode=oracle.MODE_GN, max_iter=10)
    q2, t2, log2, c2 = oracle.register_pair(P0, P1, 0.05, mode=oracle.MODE_GN, max_iter=10)
    assert ce == 0 and c == c2 and np.array_equal(q, q2) and np.array_equal(t, t2)
    assert np.array_equal(log, log2)
