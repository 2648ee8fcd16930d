"""Known-answer tests for the C++-half restatement (frameFeature / lidarOdometry_onlyPC), whose
parity against the reference binary is unpinned (it cannot be built here: ROS/PCL/Eigen/Ceres
absent).  Each case is checkable by hand from the reference source."""
import numpy as np

from helpers import frame


def test_ring_ids_at_bin_centres(oracle):
    """src/frameFeature.cpp:57-71: 64 rows -> 2 - k/3 and -8.83 - m/2; 16 rows -> -15 + 2k"""
    from ssf import synth
    for n_rows in (64, 16):
        el = np.deg2rad(synth.elevations_deg(n_rows).numpy())
        pts = np.stack([10 * np.cos(el), np.zeros_like(el), 10 * np.sin(el)], 1).astype(np.float32)
        assert np.array_equal(oracle.ring_ids(pts, n_rows), np.arange(n_rows))
    # int() truncation: 2.0 < angle < 2.5 still maps to row 0; above -> dropped
    a = np.deg2rad([2.3, 2.6, -24.5, -24.6])
    pts = np.stack([np.cos(a), np.zeros_like(a), np.sin(a)], 1).astype(np.float32)
    assert oracle.ring_ids(pts, 64).tolist() == [0, -1, 63, -1]


def test_stable_partition_and_intensity(oracle):
    pts = np.array([[10, 0, 0], [10, 0, 0.5], [10, 1, 0], [10, 0, 0.51], [10, 2, 0]], np.float32)
    rx, off, src, rid = oracle.bin_rings(pts, 16)
    # rows: angle 0 -> int((0+15)/2+0.5) = 8;  atan(0.05)=2.86deg -> int(9.43+.5)=9
    assert rid.tolist() == [8, 9, 8, 9, 8]
    assert src.tolist() == [0, 2, 4, 1, 3]           # push_back order within each row
    np.testing.assert_array_equal(rx[:, 3], np.float32([0.08, 1.08, 2.08, 0.09, 1.09]))


def test_curvature_line_and_impulse(oracle):
    """11-tap stencil: zero on evenly spaced collinear points; an offset point gives 100*d^2"""
    n = 30
    x = np.linspace(5, 8, n).astype(np.float32)
    rx = np.zeros((n, 4), np.float32)
    rx[:, 0] = 1.0
    rx[:, 1] = 2.0
    off = np.array([0] * 9 + [n] * 8, np.int64)     # all points in row 8 of 16
    cv = oracle.curvature(rx, off, 16)
    assert np.all(cv == 0)
    rx[15, 2] = 0.1
    cv = oracle.curvature(rx, off, 16)
    assert abs(cv[15] - 1.0) < 1e-6                  # (-10 * 0.1)^2
    assert abs(cv[14] - 0.01) < 1e-7                 # neighbours see 0.1^2
    assert cv[4] == 0 and cv[25] == 0                # j < 5 and j >= size-5 keep value 0
    del x


def test_greedy_selection(oracle):
    """planeSpan spacing: emit j, then skip to j + span (frameFeature.cpp:110-123)"""
    n = 20
    rx = np.zeros((n, 4), np.float32)
    rx[:, 3] = np.arange(n)
    off = np.array([0] * 9 + [n] * 8, np.int64)
    cv = np.full(n, 1.0, np.float32)
    cv[[0, 1, 2, 3, 7, 8, 9, 15, 16]] = 0.0          # candidates (value < 0.05)
    pl, sel = oracle.select(rx, cv, off, 16)         # span 3
    assert sel.tolist() == [0, 3, 7, 15]


def test_plane_fit_exact_plane(oracle):
    """points on z = -2.5: the 5x3 least squares gives n = (0, 0, +-1), all valid"""
    rng = np.random.default_rng(0)
    m = 200
    P = np.zeros((m, 4), np.float32)
    P[:, 0] = rng.uniform(0, 2, m)
    P[:, 1] = rng.uniform(0, 2, m)
    P[:, 2] = -2.5
    P[:, 3] = (np.arange(m) % 16) / 100.0 + np.arange(m)   # rows 0..15
    nrm, valid, pick, gate = oracle.plane_table(P, 0.05)
    assert valid.all()
    assert np.abs(np.abs(nrm[:, 2]) - 1).max() < 1e-6
    # gated rank: the 6th neighbour (n = 5) unless different-row points were collected
    assert set(np.unique(gate)) <= set(range(5, 30))


def test_quaternion_plus_and_accumulate(oracle):
    q, t = oracle.accumulate([0, 0, 0, 1], [1, 2, 3], [0, 0, np.sin(0.5), np.cos(0.5)], [1, 0, 0])
    # R_z(1 rad) applied to (1,0,0) after identity: t = (1,2,3) + (1,0,0)
    np.testing.assert_allclose(t, [2, 2, 3])
    q2, t2 = oracle.accumulate(q, t, [0, 0, 0, 1], [1, 0, 0])
    np.testing.assert_allclose(t2, [2 + np.cos(1.0), 2 + np.sin(1.0), 3], atol=1e-12)


def test_lm_recovers_known_transform(oracle):
    """noise-free point-to-plane correspondences generated from a known pose: LM converges to it"""
    rng = np.random.default_rng(1)
    c = 400
    nrm = rng.normal(size=(c, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    po = rng.uniform(-20, 20, (c, 3))
    ang = 0.02
    qt = np.array([0, 0, np.sin(ang / 2), np.cos(ang / 2)])
    tt = np.array([0.8, -0.1, 0.05])
    Rz = np.array([[np.cos(ang), -np.sin(ang), 0], [np.sin(ang), np.cos(ang), 0], [0, 0, 1]])
    pa = po @ Rz.T + tt + rng.normal(size=(c, 3)) * 0.0
    # move pa inside each plane (residual unchanged): pa += tangent * s
    tang = np.cross(nrm, [0, 0, 1.0])
    pa = pa + tang * rng.uniform(-0.2, 0.2, (c, 1))
    for mode, iters in ((0, 8), (1, 10)):
        q, t, log = oracle.solve(po.astype(np.float32), pa.astype(np.float32), nrm.astype(np.float32),
                                 mode=mode, max_iter=iters)
        assert np.abs(t - tt).max() < 1e-4, (mode, t)
        assert abs(abs(np.dot(q, qt)) - 1) < 1e-8


def test_oracle_register_on_synthetic_pair(oracle):
    from ssf import synth
    a = oracle.extract_planes(frame(0, 0, n_az=1875)[0], 64)
    b = oracle.extract_planes(frame(0, 1, n_az=1875)[0], 64)
    qg, tg = synth.relative_pose(0, 0, 1)
    q, t, log, c = oracle.register_pair(a, b, 0.05, q_init=qg, t_init=[tg[0] * 0.9, 0, 0])
    assert c > 100
    assert np.abs(t - np.array(tg)).max() < 0.1
    assert log.shape[0] >= 1 and np.all(np.diff(log[log[:, 8] == 1, 7]) <= 0)  # accepted steps decrease cost


# Upper-branch bin edges where `2 - angle` (frameFeature.cpp:66, int - float: a FLOAT
# subtraction) rounds across the edge that the double expression would not cross.  The z values
# put a point at x = 1, y = 0 exactly on those float angles (found by ulp search; the double
# chain of :57 lands on all three, the float chain on the first and third and on -1.5 for the
# second -- the same row).
UPPER_EDGE_CASES = [  # (z bits, float angle, row with float '2 - angle', row with double)
    (0x3C0EFB24, 0.5000000596046448, 5, 4),
    (-0x3CD683DB, -1.4999998807907104, 11, 10),
    (-0x3D32D5D0, -2.499999761581421, 14, 13),
]


def _f32_from_bits(b):
    sign = b < 0
    v = np.array([abs(b)], np.uint32).view(np.float32)[0]
    return -v if sign else v


def test_ring_id_upper_branch_float_subtraction(oracle):
    """frameFeature.cpp:66 `(2 - angle) * 3.0 + 0.5`: 2 - angle is computed and rounded in
    float, then promoted.  At these bin edges the float rounding lands on the other row."""
    for zb, ang, row_f, row_d in UPPER_EDGE_CASES:
        assert oracle.ring_id_of_angle(ang, 64) == row_f
        a32 = np.float32(ang)
        assert int(float(np.float32(2) - a32) * 3.0 + 0.5) == row_f
        assert int((2.0 - float(a32)) * 3.0 + 0.5) == row_d != row_f
        z = _f32_from_bits(zb)
        assert oracle.ring_ids(np.array([[1.0, 0.0, z]], np.float32), 64).tolist() == [row_f]
        for chain in (oracle.RING_CHAIN_FLOAT, oracle.RING_CHAIN_DOUBLE):   # both evaluations of :57
            assert oracle.lib().orc_ring_id_chain(1.0, 0.0, float(z), 64, chain) == row_f


def test_xindex_knn_equals_brute_force(oracle):
    """The oracle's x-sorted k-NN index returns the brute-force (d2, index) lists exactly,
    including exact duplicates and equal-distance ties (quantised coordinates)."""
    rng = np.random.default_rng(11)
    for trial in range(4):
        m = 700
        c = np.zeros((m, 4), np.float32)
        c[:, :3] = np.round(rng.normal(0, 3, (m, 3)) * (4 if trial % 2 else 64)) / (4 if trial % 2 else 64)
        c[rng.choice(m, 50), :3] = c[rng.choice(m, 50), :3]          # exact duplicates
        for k in (1, 5, 30):
            for qi in rng.choice(m, 40, replace=False):
                q = c[qi, :3] + (0 if qi % 3 else np.float32(0.125))
                i1, d1 = oracle.knn(c, q, k)
                i2, d2 = oracle.xknn(c, q, k)
                assert np.array_equal(i1, i2) and np.array_equal(d1, d2), (trial, k, qi)
