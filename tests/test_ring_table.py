"""The ring-id table of the feature stage (features.hip build_ring_table / ring_id_table): for every
ratio, one cell lookup + one compare must give the reference's row id (frameFeature.cpp:57-73 as
oracle/ssf_oracle.c orc_ring_angle computes it under either overload resolution):
  float chain (default): ratio z / sqrtf(r2), atanf, `* 180` in float, `/ M_PI` in double;
  double chain: ratio (double)z / sqrt((double)r2), atan and the scaling in double.
CPU only: the table is built by the library's host code; the device lookup is restated here with
the same operations (its GPU counterparts are tests/test_gpu_features.py::test_ring_id_table_edges
and ::test_ring_ids_near_bin_edges)."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ssf-slam_amd"))
CELLS = 256
CHAINS = {"float": 0, "double": 1}
NBYTES = 8 + 8 * CELLS + 2 * 4 * 64 + 8 + 8 * CELLS   # r0, inv, cells, row intervals, chain, dthr


def _raw(n_rows, chain):
    from ssf import _abi
    L = C.CDLL(_abi.LIB_PATH)
    f = getattr(L, "_ZN3ssf16build_ring_tableEiiPv")
    f.argtypes = [C.c_int, C.c_int, C.c_void_p]
    f.restype = C.c_int
    nb = getattr(L, "_ZN3ssf16ring_table_bytesEv")
    nb.restype = C.c_size_t
    assert nb() == NBYTES
    buf = (C.c_char * NBYTES)()
    assert f(n_rows, CHAINS[chain], C.addressof(buf)) == 0
    return bytes(buf)


def table(n_rows, chain="float"):
    """-> (r0, inv, cells[thr f32, ids i32], dthr f64[CELLS])"""
    raw = _raw(n_rows, chain)
    r0, inv = np.frombuffer(raw[:8], np.float32)
    cells = np.frombuffer(raw[8:8 + 8 * CELLS], np.dtype([("thr", np.float32), ("ids", np.int32)]))
    o = 8 + 8 * CELLS + 512
    assert int(np.frombuffer(raw[o:o + 4], np.int32)[0]) == CHAINS[chain]
    dthr = np.frombuffer(raw[o + 8:o + 8 + 8 * CELLS], np.float64)
    return np.float32(r0), np.float32(inv), cells, dthr


def intervals(n_rows, chain="float"):
    """per row, the [lo, hi) ratio interval of the table (the regular-window kernels' regularity check)"""
    iv = np.frombuffer(_raw(n_rows, chain)[8 + 8 * CELLS:8 + 8 * CELLS + 512], np.float32)
    return iv[:64], iv[64:]


def _cells_of(ratio_f32, r0, inv):
    ratio = np.asarray(ratio_f32, np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        tc = (ratio - r0) * inv                                    # float32 sub, mul
        ci = np.where(tc < 0, 0, np.where(tc >= CELLS, CELLS - 1, np.nan_to_num(tc, nan=0).astype(np.int64)))
    return np.clip(ci, 0, CELLS - 1)


def _ab(c):
    a = ((c["ids"] & 0xff).astype(np.int8)).astype(np.int32)
    b = (((c["ids"] >> 8) & 0xff).astype(np.int8)).astype(np.int32)
    return a, b


def lookup(ratio, r0, inv, cells):
    """the device's ring_id_lookup on float32 ratios (the float chain's exact path)"""
    ratio = np.asarray(ratio, np.float32)
    a, b = _ab(cells[_cells_of(ratio, r0, inv)])
    idv = np.where(ratio < cells[_cells_of(ratio, r0, inv)]["thr"], a, b)
    return np.where(np.isnan(ratio), -1, idv)


def lookup_d(ratio, r0, inv, cells, dthr):
    """the device's ring_id_exact on double ratios (the double chain: the cell of the float
    rounding, the cell's double threshold)"""
    ratio = np.asarray(ratio, np.float64)
    with np.errstate(over="ignore"):
        ci = _cells_of(ratio.astype(np.float32), r0, inv)
    a, b = _ab(cells[ci])
    idv = np.where(ratio < dthr[ci], a, b)
    return np.where(np.isnan(ratio), -1, idv)


def _ulps(t, dtype, k):
    it = np.int32 if dtype == np.float32 else np.int64
    u = np.asarray(t, dtype).view(it)
    return [np.asarray(u + d, it).view(dtype) for d in range(-k, k + 1)]


SPECIAL = (0.0, -0.0, np.inf, -np.inf, np.nan, 1e30, -1e30, 1e-40, -1e-40)


@pytest.mark.parametrize("n_rows", [64, 16])
def test_ring_table_equals_reference_ids_float_chain(oracle, n_rows):
    r0, inv, cells, dthr = table(n_rows, "float")
    ref = lambda r: np.array([oracle.lib().orc_ring_id_chain(1.0, 0.0, float(x), n_rows, 0) for x in r], np.int32)
    pts = [t for t in cells["thr"] if np.isfinite(t)]
    assert np.array_equal(dthr[np.isfinite(dthr)], np.array(pts, np.float64))   # the float chain's dthr = thr
    edges = [np.float32(r0 + k / inv) for k in range(CELLS + 1)]
    probe = [p for t in pts + edges for p in _ulps(np.float32(t), np.float32, 4)]
    rng = np.random.default_rng(3)
    probe += list(rng.uniform(-0.7, 0.7, 20000).astype(np.float32))
    probe += [np.float32(x) for x in SPECIAL]
    probe = np.array(probe, np.float32)
    got, want = lookup(probe, r0, inv, cells), ref(probe)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(float(probe[i]), int(got[i]), int(want[i])) for i in bad[:10]]
    assert set(want.tolist()) >= set(range(n_rows))


@pytest.mark.parametrize("n_rows", [64, 16])
def test_ring_table_float_chain_exhaustive(oracle, n_rows):
    """EVERY float ratio with 2^-12 <= |r| <= 0.7 (~2e8 floats, glibc atanf on each): the float
    chain's id changes exactly at the table's thresholds, to exactly the table's ids, and never
    back (the step function is monotone over the whole range, so bisection found every change).
    Below 2^-12 the angle is under 0.014 deg: inside row 6 for 64 rows; for 16 rows angle 0 is
    itself a bin edge ((0 + 15) / 2 + 0.5 = 8), and the table's one threshold there (where the
    float sum angle + 15 first drops below 15) is probed +-4 ulps by the float-chain test above."""
    r0, inv, cells, _ = table(n_rows, "float")
    neg_at, neg_id = oracle.ring_changes_f32(-0.7, -2.0 ** -12, n_rows)
    pos_at, pos_id = oracle.ring_changes_f32(2.0 ** -12, 0.7, n_rows)
    at = np.concatenate([neg_at[1:], pos_at[1:]])           # the first entry is the range start
    ids = np.concatenate([neg_id, pos_id])
    if n_rows == 64:
        assert neg_id[-1] == pos_id[0] == 6
        ids = np.concatenate([neg_id, pos_id[1:]])           # row 6 spans r = 0
    else:
        assert (neg_id[-1], pos_id[0]) == (7, 8)
    # rows fall as the ratio grows (64: row 0 is the top beam), rise for 16 ((angle + 15) / 2)
    d = np.diff(ids[ids >= 0])
    assert np.all(d < 0) if n_rows == 64 else np.all(d > 0)
    thr = np.sort(np.array([t for t in cells["thr"] if np.isfinite(t)], np.float32))
    inner = thr[(np.abs(thr) >= 2.0 ** -12) & (np.abs(thr) <= 0.7)]
    assert np.array_equal(np.sort(at), inner)
    tiny = thr[np.abs(thr) < 2.0 ** -12]
    assert tiny.size == (0 if n_rows == 64 else 1)
    # and the table's lookup on both sides of every change
    probe = np.array([p for t in at for p in _ulps(t, np.float32, 1)], np.float32)
    want = np.array([oracle.lib().orc_ring_id_chain(1.0, 0.0, float(x), n_rows, 0) for x in probe])
    assert np.array_equal(lookup(probe, r0, inv, cells), want)


@pytest.mark.parametrize("n_rows", [64, 16])
def test_ring_table_equals_reference_ids_double_chain(oracle, n_rows):
    """the double chain: thresholds are doubles; +-6 double ulps and +-2 float ulps around each,
    every cell edge, random and special ratios -- lookup of the double ratio == the chain's id"""
    r0, inv, cells, dthr = table(n_rows, "double")
    ref = lambda r: np.array([oracle.lib().orc_ring_id_ratio_d(float(x), n_rows) for x in r], np.int32)
    T = dthr[np.isfinite(dthr)]
    assert np.array_equal(cells["thr"][np.isfinite(dthr)], T.astype(np.float32))
    probe = [p for t in T for p in _ulps(t, np.float64, 6)]
    probe += [np.float64(p) for t in T for p in _ulps(np.float32(t), np.float32, 2)]
    probe += [np.float64(np.float32(r0 + k / inv)) for k in range(CELLS + 1)]
    rng = np.random.default_rng(5)
    probe += list(rng.uniform(-0.7, 0.7, 20000))
    probe += list(SPECIAL)
    probe = np.array(probe, np.float64)
    got, want = lookup_d(probe, r0, inv, cells, dthr), ref(probe)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(float(probe[i]), int(got[i]), int(want[i])) for i in bad[:10]]
    assert set(want.tolist()) >= set(range(n_rows))
    # exact change points: the id differs from the previous double's
    for t in T:
        assert ref([t])[0] != ref([np.nextafter(t, -np.inf)])[0]


@pytest.mark.parametrize("n_rows", [64, 16])
def test_chains_differ_only_near_bin_edges(oracle, n_rows):
    """the two chains' change points are within a few float ulps of each other (both are
    roundings of the same real thresholds), and the float chain differs from the hybrid the
    builds before round 5 used (float ratio, double atan) -- which no compilation produces"""
    _, _, cf, _ = table(n_rows, "float")
    _, _, cd, dthr = table(n_rows, "double")
    tf = np.sort(cf["thr"][np.isfinite(cf["thr"])].astype(np.float64))
    td = np.sort(dthr[np.isfinite(dthr)])
    assert tf.size == td.size
    assert np.all(np.abs(tf - td) <= 8 * np.spacing(np.abs(tf).astype(np.float32)).astype(np.float64))


@pytest.mark.parametrize("chain", ["float", "double"])
@pytest.mark.parametrize("n_rows", [64, 16])
def test_row_intervals_hold_exactly_their_row(oracle, n_rows, chain):
    """k_feat_wave_reg (and k_feat_chunk_reg) accept a point for the lane's row when its fast
    ratio lies inside the row's [lo, hi) shrunk by m = 1e-6 max(1, |lo|, |hi|): every ratio within
    4e-7 (relative: the fast ratio's error) of that shrunk interval has the row's reference id;
    float chain: lo / hi are exact (the float below lo and the float at hi are other rows)"""
    lo, hi = intervals(n_rows, chain)
    if chain == "float":
        ref = lambda x: oracle.lib().orc_ring_id_chain(1.0, 0.0, float(x), n_rows, 0)
    else:
        ref = lambda x: oracle.lib().orc_ring_id_ratio_d(float(x), n_rows)
    present = 0
    for r in range(64):
        if not lo[r] < hi[r]:
            assert r >= n_rows or not np.isfinite(lo[r])
            continue
        present += 1
        a, b = np.float32(lo[r]), np.float32(hi[r])
        if chain == "float":
            below = np.nextafter(a, np.float32(-np.inf), dtype=np.float32)
            last = np.nextafter(b, np.float32(-np.inf), dtype=np.float32)
            assert ref(a) == r and ref(last) == r and ref(below) != r and ref(b) != r, r
        m = 1e-6 * max(1.0, abs(float(a)), abs(float(b)))
        sa, sb = float(np.float32(a + np.float32(m))), float(np.float32(b - np.float32(m)))
        for x in (sa - 4e-7 * abs(sa), sa, sb, sb + 4e-7 * abs(sb)):
            assert ref(x) == r, (r, x)
        for x in np.linspace(sa, sb, 7):
            assert ref(x) == r, (r, x)
    assert present == n_rows
