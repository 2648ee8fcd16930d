"""frameFeature parity: HIP ring binning / curvature / planar selection vs the CPU oracle.

Bit-exact bar: ring ids, row offsets, the ring-ordered cloud (incl. the encoded intensity
indexInRow + row/100, src/frameFeature.cpp:77), every curvature value and the selected plane
list must be identical to the oracle (both evaluate the float expressions of
src/frameFeature.cpp:84-123 in the same order without FMA contraction).
"""
import numpy as np
import pytest
import torch

from helpers import frame, shuffled

pytestmark = pytest.mark.gpu


def _run(fe, clouds, dev, stride=3):
    import ssf
    pts = np.concatenate(clouds) if clouds else np.zeros((0, 3), np.float32)
    if stride != 3:
        pad = np.zeros((pts.shape[0], stride), np.float32)
        pad[:, :3] = pts
        pad[:, 3:] = 7.0
        pts = pad
    t = torch.from_numpy(np.ascontiguousarray(pts)).to(dev)
    off, h_off = ssf.frame_offsets([c.shape[0] for c in clouds], dev)
    return fe.extract_planes_batch(t, off, h_off, debug=True), h_off


def _check_frame(O, fe, out, h_off, f, cloud, n_rows):
    pb, ring, roff, curv = out
    rx, off_ref, _, _ = O.bin_rings(cloud, n_rows)
    cv_ref = O.curvature(rx, off_ref, n_rows)
    pl_ref, _ = O.select(rx, cv_ref, off_ref, n_rows)
    o = int(h_off[f])
    kept = int(off_ref[-1])
    assert np.array_equal(roff[f].cpu().numpy().astype(np.int64), off_ref)
    assert np.array_equal(ring[o:o + kept].cpu().numpy(), rx), "ring-ordered cloud differs"
    g = curv[o:o + kept].cpu().numpy()
    assert np.array_equal(g.view(np.uint32), cv_ref.view(np.uint32)), "curvature bits differ"
    got = pb.frame(f).cpu().numpy()
    assert got.shape == pl_ref.shape
    assert np.array_equal(got, pl_ref), "plane list differs"


@pytest.mark.parametrize("n_rows", [64, 16])
def test_single_frame_bitexact(oracle, dev, n_rows):
    import ssf
    fe = ssf.Frontend(n_rows, device=dev.index)
    cloud = frame(0, 0, n_rows=n_rows, n_az=1875)[0]
    out, h_off = _run(fe, [cloud], dev)
    _check_frame(oracle, fe, out, h_off, 0, cloud, n_rows)


def test_ragged_batch_shuffled_and_empty(oracle, dev):
    """ragged frames, arbitrary arrival order, an empty frame and a tiny frame in one batch"""
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    c0 = frame(0, 1)[0]
    c1 = shuffled(frame(1, 2)[0], 3)
    c2 = np.zeros((0, 3), np.float32)
    c3 = frame(2, 0)[0][:700]
    c4 = frame(3, 4, n_az=900)[0]
    clouds = [c0, c1, c2, c3, c4]
    out, h_off = _run(fe, clouds, dev)
    for f, c in enumerate(clouds):
        _check_frame(oracle, fe, out, h_off, f, c, 64)
    assert int(out[0].count[2]) == 0


def test_point_stride_and_dropped_rows(oracle, dev):
    """padded PCL layout (stride 4) and points outside every row (dropped, :73)"""
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    c = frame(1, 0)[0].copy()
    c[::97, 2] = 50.0       # elevation far above row 0 -> dropped
    c[1::89, 2] = -500.0    # far below row 63 -> dropped
    out, h_off = _run(fe, [c], dev, stride=4)
    _check_frame(oracle, fe, out, h_off, 0, c, 64)


def test_single_frame_api(oracle, dev):
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    c = frame(0, 3)[0]
    got = fe.extract_planes(torch.from_numpy(c).to(dev)).cpu().numpy()
    assert np.array_equal(got, oracle.extract_planes(c, 64))


def test_full_size_frame(oracle, dev):
    """BASELINE config size: 64 x 1875 = 120k points, bit-exact"""
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    c = frame(4, 7, n_az=1875)[0]
    out, h_off = _run(fe, [c, c], dev)
    _check_frame(oracle, fe, out, h_off, 1, c, 64)
