"""The synthetic scan generator's steady dynamic share (round 6) and the bench's staggered
sequence starts -- CPU only (synth.scan runs in torch on the CPU)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ssf-slam_amd"), REPO]


def test_cars_stay_in_the_window_around_the_ego():
    """Every car's centre stays in [ego + CAR_LO, ego + CAR_LO + CAR_SPAN) on every frame, and
    between two frames it moves by its velocity unless it wraps round the window."""
    from ssf import synth
    sc = synth.Scene(3)
    half = float(sc.car_half[0])
    prev = None
    for k in range(0, 400, 7):
        b = sc.car_boxes(k).numpy()
        cx = 0.5 * (b[:, 0] + b[:, 3])
        ego = k * synth.EGO_SPEED
        assert np.all(cx >= ego + sc.CAR_LO - 1e-9) and np.all(cx < ego + sc.CAR_LO + sc.CAR_SPAN + 1e-9), k
        assert np.allclose(b[:, 3] - b[:, 0], 2 * half)
        if prev is not None:
            step = cx - prev
            want = 7 * sc.cars[:, 2].numpy()
            moved = np.isclose(step, want) | np.isclose(np.abs(step - want), sc.CAR_SPAN, atol=1e-6)
            assert np.all(moved), (k, step, want)
        prev = cx


def test_late_frames_keep_dynamic_points():
    """Frames far along a sequence still carry moving-car points (before round 6 the cars drove
    out of range: no dynamic point after frame ~60, which doubled the GMM's EM iterations)."""
    from ssf import synth
    for seq, k in ((0, 0), (1, 150), (2, 300)):
        f = synth.scan(seq, k, n_az=600)
        share = float(f["s_fg_mask"].float().mean())
        assert 0.005 < share < 0.4, (seq, k, share)


def test_bench_stagger_starts():
    import argparse
    import bench
    a = argparse.Namespace(stagger=200, warmup=5, steps=20)
    st = bench.stagger_starts(a, 256)
    assert st[0] == 0 and st[1] == 7 and len(st) == 256 and max(st) < 200 and len(set(st)) == 200
    w = bench.frame_window(a, 256, 26)
    assert w["stagger"] == 200 and w["first_frame_max"] == 199 and w["timed_frames"] == [5, 25]
    a.stagger = 0
    assert bench.stagger_starts(a, 4) is None
