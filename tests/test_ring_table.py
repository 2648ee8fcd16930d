"""The ring-id table of the single-read feature stage (features.hip build_ring_table /
ring_id_table): for every float ratio, one cell lookup + one compare must give the reference's
row id (frameFeature.cpp:57-73 as oracle/ssf_oracle.c orc_ring_id computes it: float ratio,
double atan, float angle, the :60 / :63-71 bin arithmetic, int() truncation).  CPU only: the
table is built by the library's host code; the device lookup is restated here in float32 with
the same operations (its GPU counterpart is tests/test_gpu_features.py::test_ring_id_table_edges)."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ssf-slam_amd"))
CELLS = 256


def table(n_rows):
    from ssf import _abi
    L = C.CDLL(_abi.LIB_PATH)
    f = getattr(L, "_ZN3ssf16build_ring_tableEiPv")
    f.argtypes = [C.c_int, C.c_void_p]
    f.restype = C.c_int
    nb = getattr(L, "_ZN3ssf16ring_table_bytesEv")
    nb.restype = C.c_size_t
    assert nb() == 8 + 8 * CELLS + 2 * 4 * 64               # r0, inv, cells, per-row intervals
    buf = (C.c_char * nb())()
    assert f(n_rows, C.addressof(buf)) == 0
    raw = bytes(buf)
    r0, inv = np.frombuffer(raw[:8], np.float32)
    cells = np.frombuffer(raw[8:8 + 8 * CELLS], np.dtype([("thr", np.float32), ("ids", np.int32)]))
    return np.float32(r0), np.float32(inv), cells


def intervals(n_rows):
    """per row, the [lo, hi) ratio interval of the table (the regular-window kernels' regularity check)"""
    from ssf import _abi
    L = C.CDLL(_abi.LIB_PATH)
    f = getattr(L, "_ZN3ssf16build_ring_tableEiPv")
    f.argtypes = [C.c_int, C.c_void_p]
    f.restype = C.c_int
    buf = (C.c_char * (8 + 8 * CELLS + 512))()
    assert f(n_rows, C.addressof(buf)) == 0
    iv = np.frombuffer(bytes(buf)[8 + 8 * CELLS:], np.float32)
    return iv[:64], iv[64:]


def lookup(ratio, r0, inv, cells):
    """the device's ring_id_table on float32 ratios"""
    ratio = np.asarray(ratio, np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        tc = (ratio - r0) * inv                                    # float32 sub, mul
        ci = np.where(tc < 0, 0, np.where(tc >= CELLS, CELLS - 1, np.nan_to_num(tc, nan=0).astype(np.int64)))
    ci = np.clip(ci, 0, CELLS - 1)
    c = cells[ci]
    a = ((c["ids"] & 0xff).astype(np.int8)).astype(np.int32)
    b = (((c["ids"] >> 8) & 0xff).astype(np.int8)).astype(np.int32)
    idv = np.where(ratio < c["thr"], a, b)
    return np.where(np.isnan(ratio), -1, idv)


@pytest.mark.parametrize("n_rows", [64, 16])
def test_ring_table_equals_reference_ids(oracle, n_rows):
    r0, inv, cells = table(n_rows)
    ref = lambda r: np.array([oracle.lib().orc_ring_id(1.0, 0.0, float(x), n_rows) for x in r], np.int32)
    # every id change point of the table and every cell boundary, +-4 ulps around each
    pts = [t for t in cells["thr"] if np.isfinite(t)]
    edges = [np.float32(r0 + k / inv) for k in range(CELLS + 1)]
    probe = []
    for t in pts + edges:
        t = np.float32(t)
        u = t.view(np.int32)
        for d in range(-4, 5):
            probe.append(np.int32(u + d).view(np.float32))
    rng = np.random.default_rng(3)
    probe += list(rng.uniform(-0.7, 0.7, 20000).astype(np.float32))
    probe += [np.float32(x) for x in (0.0, -0.0, np.inf, -np.inf, np.nan, 1e30, -1e30, 1e-40, -1e-40)]
    probe = np.array(probe, np.float32)
    got = lookup(probe, r0, inv, cells)
    want = ref(probe)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(float(probe[i]), int(got[i]), int(want[i])) for i in bad[:10]]
    # every row appears, the change points are where the reference's id changes
    assert set(want.tolist()) >= set(range(n_rows))



@pytest.mark.parametrize("n_rows", [64, 16])
def test_row_intervals_hold_exactly_their_row(oracle, n_rows):
    """k_feat_wave_reg (and k_feat_chunk_reg) accept a point for the lane's row when its ratio lies inside the row's
    [lo, hi) with a margin: every ratio in a row's interval has that row's reference id, the
    float just below lo and the float at hi do not, and rows the profile lacks are empty"""
    lo, hi = intervals(n_rows)
    ref = lambda x: oracle.lib().orc_ring_id(1.0, 0.0, float(x), n_rows)
    present = 0
    for r in range(64):
        if not lo[r] < hi[r]:
            assert r >= n_rows or not np.isfinite(lo[r])
            continue
        present += 1
        a, b = np.float32(lo[r]), np.float32(hi[r])
        below = np.nextafter(a, np.float32(-np.inf), dtype=np.float32)
        last = np.nextafter(b, np.float32(-np.inf), dtype=np.float32)
        assert ref(a) == r and ref(last) == r and ref(below) != r and ref(b) != r, r
        for x in np.linspace(float(a), float(last), 7).astype(np.float32):
            assert ref(x) == r, (r, x)
    assert present == n_rows
