"""Pin the CPU oracle to the reference: golden vectors produced by importing the reference's
own scripts/PointCloudOdometry_noSeg.py (+ the sklearn it calls), see tests/golden/make_golden.py."""
import glob
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_mt19937_stream(oracle):
    g = np.load(os.path.join(GOLDEN, "mt19937_ref.npz"))
    for k in g.files:
        rs = oracle.LegacyRandomState(int(k[4:]))
        assert np.array_equal(rs.random_sample(8), g[k])


def test_slove_RT_by_SVD(oracle):
    g = np.load(os.path.join(GOLDEN, "kabsch_ref.npz"))
    for c in range(4):
        rc, R, t = oracle.kabsch(g[f"src{c}"], g[f"dst{c}"])
        assert rc == 0
        assert np.abs(R - g[f"R{c}"]).max() < 1e-12
        assert np.abs(t - g[f"t{c}"]).max() < 1e-12
    rc, _, _ = oracle.kabsch(g["refl_src"], g["refl_dst"])
    assert rc == -2 and int(g["refl_raises_typeerror"]) == 1


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "gmm_noseg_case*.npz"))))
def test_gmm_mask_and_pose(oracle, path):
    g = np.load(path)
    res = oracle.mask_and_pose(g["pos1"], g["flow"], g["draws"])
    info = res["info"]
    assert [int(info["center0"]), int(info["center1"])] == [int(v) for v in g["kmeans_pp_idx"]]
    assert int(info["kmeans_iter"]) == int(g["kmeans_n_iter"])
    assert int(info["em_iter"]) == int(g["gmm_n_iter"])
    assert np.array_equal(res["labels"], g["labels"])
    assert int(info["bg_label"]) == int(g["bg_label"])
    assert np.abs(res["means"] - g["gmm_means"]).max() < 1e-8
    assert abs(info["lower_bound"] - float(g["gmm_lower_bound"])) < 1e-9
    assert np.abs(res["R"] - g["R"]).max() < 1e-12
    assert np.abs(np.r_[res["t"], res["q_xyzw"]] - g["para_t_q"]).max() < 1e-12


# ASF block on float32 network output (main_sju_occ_ros.py:256-284): the reference
# fits sklearn in float32 and runs slove_RT_by_SVD on float32 arrays; this build computes the same
# block in float64 on the float32 values (a documented deviation).  Bars measured on
# the fixture (tests/golden/make_golden_asf.py): background agreement >= 99.9 % (observed
# 99.98-100 %), R within 1e-5, t within 1e-4 m (the reference's own float32 rounding: observed
# 1e-7..3e-6 and 2e-6..4e-5).  EM iteration counts may differ (f32 convergence; case 0: 18 vs 8).
ASF_BARS = dict(agree=0.999, R=1e-5, t=1e-4)


@pytest.mark.parametrize("case", range(4))
def test_asf_f32_block_deviation_bounded(oracle, case):
    g = np.load(os.path.join(GOLDEN, "gmm_asf_f32.npz"))
    assert g[f"pos1_{case}"].dtype == np.float32 and bool(g[f"means_dtype_f32_{case}"])
    res = oracle.mask_and_pose(g[f"pos1_{case}"], g[f"flow_{case}"], g[f"draws_{case}"])
    assert res["rc"] == 0
    bg_ref = (g[f"labels_{case}"] == int(g[f"bg_label_{case}"])).astype(np.uint8)
    assert (res["bg_mask"] == bg_ref).mean() >= ASF_BARS["agree"]
    assert np.abs(res["R"] - g[f"R_{case}"]).max() < ASF_BARS["R"]
    assert np.abs(res["t"] - g[f"t_{case}"]).max() < ASF_BARS["t"]
    assert not bool(g[f"quat_would_raise_{case}"])


# a19, per frame: tests/golden/make_asf_sensitivity.py refits every ASF frame with sklearn in
# float32 after 1-ulp changes of one coordinate of every k-th point.  Frames 1 and 3 are stable
# (every refit keeps the recorded EM iteration count and t bit for bit): there the float64 block
# must give the float32 reference's mask and iteration count, and its pose must be the exact
# (float64) slove_RT_by_SVD of that mask -- the remaining distance to the reference's t is the
# reference's own float32 Kabsch rounding (up to 1.5e-5 m on frame 3; the float32 restatement
# oracle.kabsch_f32 closes it: test_asf_kabsch_f32_restatement below).  On frames 0 and 2 the float32 fit itself is not
# determined beyond its rounding (refits: n_iter 6..15 / 12..13, t moved by up to 7e-5 /
# 4e-4 m): there the deviation must stay inside that spread.
def asf_case_bars(case):
    s = np.load(os.path.join(GOLDEN, "asf_f32_sensitivity.npz"))
    g = np.load(os.path.join(GOLDEN, "gmm_asf_f32.npz"))
    n0 = int(g[f"n_iter_{case}"])
    iters = [n0] + [int(v) for v in s[f"n_iter_{case}"]]
    return dict(stable=bool(s[f"stable_{case}"]), n_iter=n0, n_lo=min(iters), n_hi=max(iters),
                t_spread=float(s[f"t_spread_{case}"]), agree=float(s[f"bg_agree_{case}"].min()))


def asf_check(case, bg_mask, em_iter, t):
    """the per-frame a19 bars for one device / oracle result"""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle.cpu_leg import kabsch_np
    g = np.load(os.path.join(GOLDEN, "gmm_asf_f32.npz"))
    b = asf_case_bars(case)
    P, F = g[f"pos1_{case}"], g[f"flow_{case}"]
    bg_ref = (g[f"labels_{case}"] == int(g[f"bg_label_{case}"])).astype(np.uint8)
    dt = np.abs(np.asarray(t) - g[f"t_{case}"]).max()
    if b["stable"]:
        assert np.array_equal(np.asarray(bg_mask), bg_ref), case
        assert int(em_iter) == b["n_iter"], case
        m = bg_ref != 0
        _, t64 = kabsch_np((P[m] + F[m]).astype(np.float64), P[m].astype(np.float64))
        t64 = np.asarray(t64).ravel()
        assert np.abs(np.asarray(t) - t64).max() < 1e-6, case               # the exact Kabsch
        assert dt <= np.abs(t64 - g[f"t_{case}"]).max() + 1e-6, case          # = f32 rounding
    else:
        assert b["n_lo"] <= int(em_iter) <= b["n_hi"], case
        assert dt <= b["t_spread"], case
        assert (np.asarray(bg_mask) == bg_ref).mean() >= b["agree"], case


@pytest.mark.parametrize("case", range(4))
def test_asf_f32_per_frame_against_float32_sensitivity(oracle, case):
    g = np.load(os.path.join(GOLDEN, "gmm_asf_f32.npz"))
    res = oracle.mask_and_pose(g[f"pos1_{case}"], g[f"flow_{case}"], g[f"draws_{case}"])
    asf_check(case, res["bg_mask"], res["info"]["em_iter"], res["t"])


# a19 float32 tail: slove_RT_by_SVD + Quaternion restated on float32 arrays
# (oracle/ssf_oracle.c orc_kabsch_f32, main_sju_occ_ros.py:273-284,455-473).  Given the fixture's
# own labels it reproduces the reference's float32 R and t to the last bits the unpinned sgemm /
# sgesdd orders leave (observed R <= 2.1e-7, t <= 3.0e-7 m); the bar is 1e-6.
F32_TAIL_BAR = dict(R=1e-6, t=1e-6)


@pytest.mark.parametrize("case", range(4))
def test_asf_kabsch_f32_restatement(oracle, case):
    g = np.load(os.path.join(GOLDEN, "gmm_asf_f32.npz"))
    bg = (g[f"labels_{case}"] == int(g[f"bg_label_{case}"])).astype(np.uint8)
    rc, R, t, q = oracle.kabsch_f32(g[f"pos1_{case}"], g[f"flow_{case}"], bg)
    assert rc == 0 and not bool(g[f"quat_would_raise_{case}"])
    assert np.abs(R - g[f"R_{case}"]).max() < F32_TAIL_BAR["R"]
    assert np.abs(t - g[f"t_{case}"]).max() < F32_TAIL_BAR["t"]
    # q is the rotation of R (pyquaternion trace method on the f32 R)
    x, y, z, w = q
    Rq = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                   [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                   [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    assert np.abs(Rq - R).max() < 1e-6


def test_kabsch_f32_sequential_mean_and_reflection(oracle):
    """the f32 means are numpy's: add.reduce over axis 0 accumulates row after row in float32"""
    rng = np.random.default_rng(7)
    P = (rng.standard_normal((5000, 3)) * 30).astype(np.float32)
    F = (rng.standard_normal((5000, 3)) * 0.01 + 0.5).astype(np.float32)
    m = (rng.random(5000) < 0.9).astype(np.uint8)
    rc, R, t, _ = oracle.kabsch_f32(P, F, m)
    src, dst = (P + F)[m != 0], P[m != 0]
    sm, dm = src.mean(axis=0), dst.mean(axis=0)
    assert sm.dtype == np.float32
    assert np.array_equal(np.cumsum(src, axis=0, dtype=np.float32)[-1] / np.float32(len(src)), sm)
    U, S, Vt = np.linalg.svd((src - sm).T @ (dst - dm))
    Rn = Vt.T @ U.T
    assert rc == 0 and np.abs(R - Rn).max() < 1e-6
    assert np.abs(t - (-Rn @ sm + dm)).max() < 1e-5
    rc, _, _, _ = oracle.kabsch_f32(P, F, np.zeros(5000, np.uint8))
    assert rc == -1
    rc, _, _, _ = oracle.kabsch_f32(P, -2 * P, None)          # src = -dst: a reflection
    assert rc == -2


@pytest.mark.parametrize("case", range(4))
def test_asf_f32_tail_per_frame(oracle, case):
    """GMM (f64 on the f32 values) + the float32 tail: on the stable frames the reference's mask
    and EM count, and R / t within 1e-6 of the reference's float32 result (VERDICT r3 a19 'done'
    bar); on the unstable frames inside the float32 refits' spread."""
    g = np.load(os.path.join(GOLDEN, "gmm_asf_f32.npz"))
    res = oracle.mask_and_pose(g[f"pos1_{case}"], g[f"flow_{case}"], g[f"draws_{case}"],
                               kabsch_dtype="float32")
    assert res["rc"] == 0
    b = asf_case_bars(case)
    bg_ref = (g[f"labels_{case}"] == int(g[f"bg_label_{case}"])).astype(np.uint8)
    if b["stable"]:
        assert np.array_equal(res["bg_mask"], bg_ref)
        assert int(res["info"]["em_iter"]) == b["n_iter"]
        assert np.abs(res["R"] - g[f"R_{case}"]).max() < F32_TAIL_BAR["R"]
        assert np.abs(res["t"] - g[f"t_{case}"]).max() < F32_TAIL_BAR["t"]
    else:
        assert np.abs(res["t"] - g[f"t_{case}"]).max() <= b["t_spread"]
