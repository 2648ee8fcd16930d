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


def test_chunk_and_scan_boundaries(oracle, dev):
    """frames cut at the binning chunk (kBinChunk = 2048 points, ssf_internal.hpp) and at the
    scan's 16-chunk batches (k_bin_scan): 2047 / 2048 / 16 x 2048 +- 1 / 32 x 2048 points, in one
    ragged batch (every frame scans the batch's chunk count), bit-exact"""
    import ssf
    fe = ssf.Frontend(64, device=dev.index)
    full = frame(4, 7, n_az=1875)[0]
    sizes = [2047, 2048, 16 * 2048 - 1, 16 * 2048, 16 * 2048 + 1, 32 * 2048]
    clouds = [full[:n] for n in sizes]
    out, h_off = _run(fe, clouds, dev)
    for f, c in enumerate(clouds):
        _check_frame(oracle, fe, out, h_off, f, c, 64)


@pytest.mark.parametrize("n_rows,n_az", [(16, 2047), (16, 2048), (16, 2049), (16, 4500), (64, 4097)])
def test_rows_across_curvature_tiles(oracle, dev, n_rows, n_az):
    """k_bin_curv works on 2048-point input chunks with a halo of input points (a row spans
    several chunks, a chunk several rows) and k_select walks each row's candidate words: rows of
    one chunk exactly, one point over, 2-3 chunks, and the 16-beam span (3) whose selections cross
    every chunk and word edge; curvature bits and plane lists bit-exact vs the oracle"""
    import ssf
    fe = ssf.Frontend(n_rows, device=dev.index)
    c = frame(5, 1, n_rows=n_rows, n_az=n_az)[0]
    out, h_off = _run(fe, [c[: len(c) // 2], c], dev)
    _check_frame(oracle, fe, out, h_off, 0, c[: len(c) // 2], n_rows)
    _check_frame(oracle, fe, out, h_off, 1, c, n_rows)


@pytest.mark.parametrize("chain", ["float", "double"])
@pytest.mark.parametrize("n_rows", [16, 64])
def test_ring_ids_near_bin_edges(oracle, dev, n_rows, chain):
    """Elevations on and within 1e-6..1e-2 deg of every bin edge (and the -8.83 switch), plus a
    uniform spread, under both evaluations of src/frameFeature.cpp:57 (ssf_config.ring_chain:
    the float overloads, the default, and the all-double chain): the table's fast ratio must
    defer to the exact ratio wherever the two could disagree, so the binned cloud is
    bit-identical to the oracle's under the same chain."""
    import ssf
    O = oracle
    if n_rows == 64:
        edges = [2.0 - (k - 0.5) / 3.0 for k in range(-2, 35)] + [-8.83] + \
                [-8.83 - (m - 0.5) / 2.0 for m in range(0, 34)]
    else:
        edges = [-15.0 + 2.0 * k - 1.0 for k in range(0, 18)]
    rng = np.random.default_rng(7)
    el = []
    for e in edges:
        for d in (0.0, 1e-6, -1e-6, 1e-5, -1e-5, 1e-4, -1e-4, 5e-4, -5e-4, 2e-3, -2e-3, 1e-2, -1e-2):
            el.append(e + d)
    el = np.array(el + list(rng.uniform(-32.0, 12.0, 20000)), np.float64)
    az = rng.uniform(0, 2 * np.pi, el.size)
    rng_m = rng.uniform(2.0, 90.0, el.size)
    e = np.radians(el)
    pts = np.stack([rng_m * np.cos(e) * np.cos(az), rng_m * np.cos(e) * np.sin(az),
                    rng_m * np.sin(e)], 1).astype(np.float32)
    fe = ssf.Frontend(n_rows, device=dev.index or 0, ring_chain=chain)
    out, h_off = _run(fe, [pts], dev)
    pb, ring, roff, curv = out
    with O.ring_chain(chain):
        rx, off_ref, _, rid = O.bin_rings(pts, n_rows)
    assert np.array_equal(roff[0].cpu().numpy().astype(np.int64), off_ref)
    kept = int(off_ref[-1])
    assert np.array_equal(ring[:kept].cpu().numpy(), rx), "ring-ordered cloud differs near bin edges"
    other = [O.lib().orc_ring_id_chain(float(p[0]), float(p[1]), float(p[2]), n_rows,
                                       O.RING_CHAINS["double" if chain == "float" else "float"]) for p in pts]
    # the set holds points the two chains bin differently (64 rows: 25, 16 rows: 3), so a device
    # that ignored ring_chain would fail one of the two parametrisations
    assert np.count_nonzero(np.array(other) != rid) > 0


def test_mask_before_features_equals_compacted_cloud(oracle, dev):
    """Beyond the reference (BASELINE configs[2], flag off by default): extraction from the kept
    points only equals the reference extraction of the stably compacted cloud -- with the
    ground-truth background mask and with a random mask, two frames in one batch."""
    import ssf
    from helpers import frame as fr
    O = oracle
    rng = np.random.default_rng(11)
    clouds, keeps = [], []
    for k in range(2):
        pts, _, fg = fr(2, k)
        clouds.append(pts)
        keeps.append((fg == 0).astype(np.uint8) if k == 0 else (rng.random(pts.shape[0]) < 0.8).astype(np.uint8))
    fe = ssf.Frontend(64, device=dev.index or 0)
    t = torch.from_numpy(np.concatenate(clouds)).to(dev)
    keep = torch.from_numpy(np.concatenate(keeps)).to(dev)
    off, h_off = ssf.frame_offsets([c.shape[0] for c in clouds], dev)
    pb = fe.extract_planes_batch(t, off, h_off, keep=keep)
    torch.cuda.synchronize()
    for f in range(2):
        ref = O.extract_planes(clouds[f][keeps[f] != 0], 64)
        got = pb.frame(f).cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), f


def test_ring_id_upper_branch_float_subtraction(oracle, dev):
    """frameFeature.cpp:66 `(2 - angle)` is a float subtraction: at these bin edges its
    rounding picks the other row than a double subtraction would (known-answer cases shared with
    tests/test_oracle_known.py); the device rows equal the oracle's."""
    import ssf
    from test_oracle_known import UPPER_EDGE_CASES, _f32_from_bits
    pts = np.array([[1.0, 0.0, _f32_from_bits(zb)] for zb, _, _, _ in UPPER_EDGE_CASES], np.float32)
    pts = np.concatenate([pts, frame(0, 0)[0]])
    fe = ssf.Frontend(64, device=dev.index or 0)
    out, h_off = _run(fe, [pts], dev)
    pb, ring, roff, curv = out
    rx, off_ref, src, rid = oracle.bin_rings(pts, 64)
    assert rid[:3].tolist() == [c[2] for c in UPPER_EDGE_CASES]
    assert np.array_equal(roff[0].cpu().numpy().astype(np.int64), off_ref)
    kept = int(off_ref[-1])
    assert np.array_equal(ring[:kept].cpu().numpy(), rx)


def test_masked_rows_with_0_1_2_points(oracle, dev):
    """Rows in range left with 0, 1, 2, 3 and 11 points by the keep mask (a GMM that splits a frame
    badly does this, BASELINE configs[2]): a one-point row selects its only point, which is also its
    last slot -- the selection stores of the other lanes must not land there.  Bit-exact vs the
    oracle on the compacted cloud, masked and as an unmasked cloud with the same rows."""
    import ssf
    pts = frame(0, 0, n_az=600)[0]
    rid = oracle.ring_ids(pts, 64)
    keep = np.ones(len(pts), np.uint8)
    for row, n in [(8, 0), (9, 1), (10, 2), (11, 3), (12, 11), (13, 1), (57, 1), (58, 2)]:
        idx = np.nonzero(rid == row)[0]
        keep[idx[n:]] = 0
    fe = ssf.Frontend(64, device=dev.index or 0)
    t = torch.from_numpy(np.concatenate([pts, pts])).to(dev)
    k2 = torch.from_numpy(np.concatenate([keep, keep])).to(dev)
    off, h_off = ssf.frame_offsets([len(pts), len(pts)], dev)
    pb = fe.extract_planes_batch(t, off, h_off, keep=k2)
    ref = oracle.extract_planes(pts[keep != 0], 64)
    for f in range(2):
        assert np.array_equal(pb.frame(f).cpu().numpy().view(np.uint32), ref.view(np.uint32)), f
    out, h2 = _run(fe, [pts[keep != 0]], dev)
    _check_frame(oracle, fe, out, h2, 0, pts[keep != 0], 64)


def _planes_product(fe, clouds, dev):
    """the product path (no debug outputs: k_bin_curv<false> / k_curv_fixup<false>)"""
    import ssf
    t = torch.from_numpy(np.ascontiguousarray(np.concatenate(clouds))).to(dev)
    off, h_off = ssf.frame_offsets([c.shape[0] for c in clouds], dev)
    pb = fe.extract_planes_batch(t, off, h_off)
    return [pb.frame(f).cpu().numpy() for f in range(len(clouds))]


def test_curvature_halo_and_fixup_orders(oracle, dev):
    """k_bin_curv reads a stencil from its window (the chunk +- 384 input points) when the row
    has 5 points on each side there, and leaves the rest to k_curv_fixup (taps through the ring
    index).  Input orders that exercise every case: azimuth order with whole azimuth columns
    missing in some rows (sparse rows: a few stencils open), row-major order (a chunk is one or
    two rows: every stencil in the window), a fully shuffled frame (almost every stencil open),
    and a frame whose first half is shuffled.  Debug outputs (curvature bits, ring cloud) and the
    product path's plane lists, bit-exact vs the oracle."""
    import ssf
    O = oracle
    base = frame(6, 2, n_az=1875)[0]
    rid = O.ring_ids(base, 64)
    rng = np.random.default_rng(5)
    # sparse rows: rows 20..27 keep only 1 azimuth column in 9 (a row point every ~576 inputs)
    drop = np.isin(rid, np.arange(20, 28)) & (rng.random(len(base)) < 8 / 9)
    sparse = base[~drop]
    rowmajor = base[np.argsort(rid, kind="stable")]
    half = base.copy()
    half[: len(half) // 2] = shuffled(half[: len(half) // 2], 9)
    clouds = [sparse, rowmajor, shuffled(base, 4), half]
    fe = ssf.Frontend(64, device=dev.index or 0)
    out, h_off = _run(fe, clouds, dev)
    for f, c in enumerate(clouds):
        _check_frame(O, fe, out, h_off, f, c, 64)
    got = _planes_product(fe, clouds, dev)
    for f, c in enumerate(clouds):
        assert np.array_equal(got[f].view(np.uint32), O.extract_planes(c, 64).view(np.uint32)), f


def test_product_path_equals_debug_path(oracle, dev):
    """the product instantiation (no ring cloud, no curvature out) selects the same planes as the
    debug one, on a full 120k-point frame and a 16-beam frame, bit for bit (and both = oracle)"""
    import ssf
    for n_rows, n_az in [(64, 1875), (16, 4500)]:
        c = frame(7, 3, n_rows=n_rows, n_az=n_az)[0]
        fe = ssf.Frontend(n_rows, device=dev.index or 0)
        got = _planes_product(fe, [c, c[: len(c) // 3]], dev)
        assert np.array_equal(got[0].view(np.uint32), oracle.extract_planes(c, n_rows).view(np.uint32))
        assert np.array_equal(got[1].view(np.uint32), oracle.extract_planes(c[: len(c) // 3], n_rows).view(np.uint32))


@pytest.mark.parametrize("chain", ["float", "double"])
@pytest.mark.parametrize("n_rows", [64, 16])
def test_ring_id_table_edges(oracle, dev, n_rows, chain):
    """The single-read stage's ring id (one table cell + one compare, features.hip
    ring_id_table) on the exact ratios where the reference's row id changes, +-3 ulps around each
    (points (1, 0, ratio): z / sqrt(1) is the ratio itself in both chains), every cell edge, the
    origin (0/0) and +-inf ratios: the ring-ordered cloud equals the oracle's under the same
    evaluation of frameFeature.cpp:57 (glibc atanf / atan), so every point lands in the
    reference's row.  The points are shuffled and 64 copies of each are interleaved, so every
    row holds enough points for full stencils as well."""
    import ssf
    import test_ring_table as rt
    r0, inv, cells, _ = rt.table(n_rows, chain)
    probe = []
    for t in [t for t in cells["thr"] if np.isfinite(t)] + [np.float32(r0 + k / inv) for k in range(0, 257, 8)]:
        u = np.float32(t).view(np.int32)
        probe += [np.int32(u + d).view(np.float32) for d in range(-3, 4)]
    z = np.array(probe, np.float32)
    pts = np.stack([np.ones_like(z), np.zeros_like(z), z], 1)
    pts = np.concatenate([pts, [[0, 0, 0], [0, 0, 1], [0, 0, -1]]]).astype(np.float32)
    rng = np.random.default_rng(n_rows)
    cloud = np.concatenate([pts[rng.permutation(len(pts))] for _ in range(64)]).astype(np.float32)
    fe = ssf.Frontend(n_rows, device=dev.index, ring_chain=chain)
    out, h_off = _run(fe, [cloud], dev)
    with oracle.ring_chain(chain):
        _check_frame(oracle, fe, out, h_off, 0, cloud, n_rows)
        ids = np.array([oracle.lib().orc_ring_id(float(p[0]), float(p[1]), float(p[2]), n_rows) for p in pts])
    assert len(set(ids.tolist()) - {-1}) == n_rows         # every row is exercised


def test_frames_above_single_read_capacity(oracle, dev):
    """k_feat_select holds a frame's chunk counts for at most kFeatMaxChunks = 128 chunks
    (262 144 points); a launch whose frames may be larger takes the round-3 kernels
    (k_bin_count / k_bin_scan / k_bin_curv / k_select, features.hip launch_extract_planes).  A
    64 x 4200 = 268 800-point frame, the same frame shuffled, and a short one in the same launch:
    ring cloud, curvature bits and plane lists bit-exact, debug and product instantiations."""
    import ssf
    c = frame(8, 2, n_az=4200)[0]
    assert c.shape[0] > 128 * 2048
    clouds = [c, shuffled(c, 3), c[:5000]]
    fe = ssf.Frontend(64, device=dev.index or 0)
    out, h_off = _run(fe, clouds, dev)
    for f, cl in enumerate(clouds):
        _check_frame(oracle, fe, out, h_off, f, cl, 64)
    got = _planes_product(fe, clouds, dev)
    for f, cl in enumerate(clouds):
        assert np.array_equal(got[f].view(np.uint32), oracle.extract_planes(cl, 64).view(np.uint32)), f


def test_regular_windows_mixed_with_flagged_blocks(oracle, dev):
    """k_feat_wave_reg (k_feat_chunk_reg in the A/B build) does the windows of an azimuth-ordered 64-beam scan (whole columns, every
    row once per column, one row per lane) and flags every other block for k_feat_chunk;
    k_feat_select then mixes lane-map positions and u16-index positions in one frame.  A full
    120k-point frame with a NaN point (no row) in one chunk, a point moved to another ring in a
    second, and a column's two points swapped in a third -- those windows (and their neighbours'
    halos) go through the general kernel -- next to the clean frame and a frame cut mid-column
    (a ragged last window): ring cloud, curvature bits and plane lists bit-exact vs the oracle,
    debug and product instantiations."""
    import ssf
    c = frame(9, 5, n_az=1875)[0]
    d = c.copy()
    d[10 * 2048 + 700] = np.nan                               # no row
    d[30 * 2048 + 1000, 2] += 3.0                             # another ring
    i = 45 * 2048 + 64 * 7 + 3
    d[[i, i + 1]] = d[[i + 1, i]]                             # lane order broken in one column
    clouds = [c, d, c[: 64 * 1000 + 17]]
    fe = ssf.Frontend(64, device=dev.index or 0)
    out, h_off = _run(fe, clouds, dev)
    for f, cl in enumerate(clouds):
        _check_frame(oracle, fe, out, h_off, f, cl, 64)
    got = _planes_product(fe, clouds, dev)
    for f, cl in enumerate(clouds):
        assert np.array_equal(got[f].view(np.uint32), oracle.extract_planes(cl, 64).view(np.uint32)), f


def test_outermost_window_columns_not_loaded(oracle, dev):
    """k_feat_wave_reg loads a chunk's 32 own columns and 5 on each side, not the window's
    outermost column on each side (6 halo columns): no own stencil reaches it, and it cannot change
    whether one is covered.  Points broken exactly there -- a NaN (no row) in window column 0 of
    chunk 20, a point moved to another ring in window column 43 of chunk 40, two lanes swapped in
    window column 0 of chunk 50 -- make the neighbouring chunk (whose own column it is) irregular,
    while the chunk itself stays on the regular path; one more break in window column 1 of chunk
    30 (a loaded column) flags both.  Ring cloud, curvature bits and plane lists bit-exact vs the
    oracle, debug and product instantiations, for even (left-to-right) and odd (right-to-left)
    chunks."""
    import ssf
    c = frame(11, 3, n_az=1875)[0]
    d = c.copy()
    col = lambda k: 64 * k                                    # first input of global column k
    d[col(20 * 32 - 6) + 9] = np.nan                          # chunk 20, window column 0
    d[col(40 * 32 + 32 + 5) + 17, 2] += 3.0                   # chunk 40, window column 43
    i = col(50 * 32 - 6) + 30
    d[[i, i + 1]] = d[[i + 1, i]]                             # chunk 50, window column 0
    d[col(30 * 32 - 5) + 40] = np.nan                         # chunk 30, window column 1
    e = c.copy()                                              # odd chunks: 21 (column 0), 41 (43)
    e[col(21 * 32 - 6) + 3, 2] -= 2.5
    e[col(41 * 32 + 32 + 5) + 60] = np.nan
    clouds = [d, e, c]
    fe = ssf.Frontend(64, device=dev.index or 0)
    out, h_off = _run(fe, clouds, dev)
    for f, cl in enumerate(clouds):
        _check_frame(oracle, fe, out, h_off, f, cl, 64)
    got = _planes_product(fe, clouds, dev)
    for f, cl in enumerate(clouds):
        assert np.array_equal(got[f].view(np.uint32), oracle.extract_planes(cl, 64).view(np.uint32)), f


def test_carla_layout_frames(oracle, dev):
    """The reference's own data layout (ssf/synth.py layout "carla": channel-major as CARLA stores
    a sweep, no-return rays and road points dropped, random drop-off; rows ragged, several empty):
    two full 120k-point frames and a cut one in one launch -- ring cloud, curvature bits and plane
    lists bit-exact vs the oracle, debug and product instantiations, both ring-id chains."""
    import ssf
    from ssf import synth
    sc = synth.Scene(12)
    c0 = synth.scan(12, 0, n_az=1875, scene=sc, layout="carla")["pos1"].numpy()
    c1 = synth.scan(12, 1, n_az=1875, scene=sc, layout="carla")["pos1"].numpy()
    clouds = [c0, c1, c1[: 64 * 700 + 33]]
    for chain in ("float", "double"):
        fe = ssf.Frontend(64, device=dev.index or 0, ring_chain=chain)
        out, h_off = _run(fe, clouds, dev)
        with oracle.ring_chain(chain):
            for f, cl in enumerate(clouds):
                _check_frame(oracle, fe, out, h_off, f, cl, 64)
            got = _planes_product(fe, clouds, dev)
            for f, cl in enumerate(clouds):
                assert np.array_equal(got[f].view(np.uint32), oracle.extract_planes(cl, 64).view(np.uint32)), f


def test_run_kernel_orders_gaps_and_fallbacks(oracle, dev):
    """k_feat_wave_run's cases (features.hip): rows in DESCENDING order (own-tile slots are not the
    input order: the bit planes move run by run), points in no row between runs (gaps) and inside
    a run (the row then forms two runs in a chunk: left to k_feat_chunk), rows alternating in
    100-point blocks (a row in several runs per chunk: fallback), many short runs (> 64 runs in a
    chunk: fallback), a 16-beam channel-major frame, and masked frames (keep: every masked point
    is a gap).  Ring cloud, curvature bits and plane lists bit-exact vs the oracle, debug and
    product instantiations."""
    import ssf
    from ssf import synth
    sc = synth.Scene(13)
    base = synth.scan(13, 2, n_az=1875, scene=sc, layout="carla")["pos1"].numpy()
    rid = oracle.ring_ids(base, 64)
    desc = base[np.argsort(-rid, kind="stable")]                        # rows descending
    gaps = base.copy()
    gaps[5000:5003] = np.nan                                            # inside a run: two runs
    gaps[np.nonzero(np.diff(rid) != 0)[0][:6] + 1] = np.nan             # at run starts: gaps
    rowmajor = base[np.argsort(rid, kind="stable")]
    blocks = []                                                         # rows 10 / 11 alternating
    r10, r11 = rowmajor[rid[np.argsort(rid, kind="stable")] == 10], rowmajor[rid[np.argsort(rid, kind="stable")] == 11]
    for i in range(0, min(len(r10), len(r11)), 100):
        blocks += [r10[i:i + 100], r11[i:i + 100]]
    alt = np.concatenate(blocks + [rowmajor[:20000]])
    short = np.concatenate([rowmajor[rid[np.argsort(rid, kind="stable")] == r][:12] for r in range(56)] * 20)
    clouds = [desc, gaps, alt, short]
    fe = ssf.Frontend(64, device=dev.index or 0)
    out, h_off = _run(fe, clouds, dev)
    for f, cl in enumerate(clouds):
        _check_frame(oracle, fe, out, h_off, f, cl, 64)
    got = _planes_product(fe, clouds, dev)
    for f, cl in enumerate(clouds):
        assert np.array_equal(got[f].view(np.uint32), oracle.extract_planes(cl, 64).view(np.uint32)), f
    # 16 beams, channel-major
    c16 = synth.scan(14, 1, n_rows=16, n_az=4000, layout="carla")["pos1"].numpy()
    fe16 = ssf.Frontend(16, device=dev.index or 0)
    out, h_off = _run(fe16, [c16], dev)
    _check_frame(oracle, fe16, out, h_off, 0, c16, 16)
    assert np.array_equal(_planes_product(fe16, [c16], dev)[0].view(np.uint32),
                          oracle.extract_planes(c16, 16).view(np.uint32))
    # masked: a random mask and a mask of contiguous blocks
    rng = np.random.default_rng(9)
    k1 = (rng.random(len(base)) < 0.9).astype(np.uint8)
    k2 = np.ones(len(base), np.uint8)
    for s0 in range(3000, len(base), 20000):
        k2[s0:s0 + 700] = 0
    t = torch.from_numpy(np.concatenate([base, base])).to(dev)
    keep = torch.from_numpy(np.concatenate([k1, k2])).to(dev)
    off, h2 = ssf.frame_offsets([len(base), len(base)], dev)
    pb = fe.extract_planes_batch(t, off, h2, keep=keep)
    for f, kk in enumerate((k1, k2)):
        ref = oracle.extract_planes(base[kk != 0], 64)
        assert np.array_equal(pb.frame(f).cpu().numpy().view(np.uint32), ref.view(np.uint32)), f
