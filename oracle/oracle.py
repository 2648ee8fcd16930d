"""ctypes wrapper around oracle/build/libssf_oracle.so -- the CPU restatement of the
SSF-SLAM front-end hot path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the parity checker / CPU baseline.  The product package
(ssf-slam_amd/ssf) never imports this module.

Parity status: the Python half (GMM mask, Kabsch, quaternion) is pinned against golden
vectors generated from the reference's own scripts/PointCloudOdometry_noSeg.py; the C++ half
(frameFeature.cpp / lidarOdometry_onlyPC.cpp) is PARITY UNPINNED against the reference
binary (ROS/PCL/Eigen/Ceres are absent, so it cannot be built) and is pinned only by
known-answer tests.  See oracle/ssf_oracle.h and DESIGN.md.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libssf_oracle.so")
_lib = None

f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")

LOG_STRIDE = 10
MODE_CERES_LM = 0
MODE_GN = 1


class Profile(C.Structure):
    _fields_ = [("n_rows", C.c_int32), ("plane_min", C.c_float), ("plane_span", C.c_int32),
                ("row_start", C.c_int32), ("row_end", C.c_int32), ("plane_max", C.c_float)]


class IcpParams(C.Structure):
    _fields_ = [("max_iter", C.c_int32), ("max_corr_dist", C.c_float), ("trans_eps", C.c_double),
                ("fit_eps", C.c_double)]


class IcpResult(C.Structure):
    _fields_ = [("T", C.c_float * 16), ("fitness", C.c_double), ("converged", C.c_int32),
                ("iterations", C.c_int32), ("state", C.c_int32), ("n_corr", C.c_int32)]


ICP_STATES = {0: "not_converged", 1: "iterations", 2: "transform", 3: "abs_mse", 4: "rel_mse",
              5: "no_correspondences"}


def build():
    """Compile the oracle with its committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    L = C.CDLL(_LIB_PATH)
    L.orc_profile_get.argtypes = [C.c_int32, C.POINTER(Profile)]
    L.orc_ring_id.argtypes = [C.c_float, C.c_float, C.c_float, C.c_int32]
    L.orc_ring_id.restype = C.c_int32
    L.orc_ring_id_of_angle.argtypes = [C.c_float, C.c_int32]
    L.orc_ring_id_of_angle.restype = C.c_int32
    L.orc_set_ring_chain.argtypes = [C.c_int32]
    L.orc_set_ring_chain.restype = C.c_int32
    L.orc_get_ring_chain.restype = C.c_int32
    L.orc_ring_angle.argtypes = [C.c_float, C.c_float, C.c_float, C.c_int32]
    L.orc_ring_angle.restype = C.c_float
    L.orc_ring_id_chain.argtypes = [C.c_float, C.c_float, C.c_float, C.c_int32, C.c_int32]
    L.orc_ring_id_chain.restype = C.c_int32
    L.orc_ring_id_ratio_d.argtypes = [C.c_double, C.c_int32]
    L.orc_ring_id_ratio_d.restype = C.c_int32
    L.orc_ring_changes_f32.argtypes = [C.c_float, C.c_float, C.c_int32, f32p, i32p, C.c_int64]
    L.orc_ring_changes_f32.restype = C.c_int64
    L.orc_xindex_build.argtypes = [C.c_void_p, C.c_int64]
    L.orc_xindex_build.restype = C.c_void_p
    L.orc_xindex_free.argtypes = [C.c_void_p]
    L.orc_xindex_knn.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
    L.orc_bin.argtypes = [f32p, C.c_int64, C.c_int64, C.c_int32, f32p, i64p, i64p, i32p]
    L.orc_bin.restype = C.c_int64
    L.orc_curvature.argtypes = [f32p, i64p, C.c_int32, C.c_int32, C.c_int32, f32p]
    L.orc_select.argtypes = [f32p, f32p, i64p, C.c_int32, C.c_int32, C.c_int32, C.c_float,
                             C.c_int32, f32p, i64p]
    L.orc_select.restype = C.c_int64
    L.orc_extract_planes.argtypes = [f32p, C.c_int64, C.c_int64, C.c_int32, f32p]
    L.orc_extract_planes.restype = C.c_int64
    L.orc_knn.argtypes = [f32p, C.c_int64, f32p, C.c_int32, i32p, f32p]
    L.orc_plane_table.argtypes = [f32p, C.c_int64, C.c_float, f32p, i32p, i32p, i32p]
    L.orc_transform_point.argtypes = [f64p, f64p, f32p, f32p]
    L.orc_correspond.argtypes = [f32p, C.c_int64, f32p, C.c_int64, f64p, f64p, i32p]
    L.orc_solve.argtypes = [f32p, f32p, f32p, C.c_int64, C.c_int32, C.c_int32, f64p, f64p, f64p,
                            f64p, f64p, C.POINTER(C.c_int32)]
    L.orc_solve.restype = C.c_int32
    L.orc_register_pair.argtypes = [f32p, C.c_int64, f32p, C.c_int64, C.c_float, C.c_int32,
                                    C.c_int32, f64p, f64p, f64p, f64p, f64p, C.POINTER(C.c_int32)]
    L.orc_register_pair.restype = C.c_int64
    L.orc_accumulate.argtypes = [f64p, f64p, f64p, f64p, f64p, f64p]
    L.orc_select_edges.argtypes = [f32p, f32p, i64p, C.c_int32, C.c_int32, C.c_int32, C.c_float,
                                   C.c_int32, f32p]
    L.orc_select_edges.restype = C.c_int64
    L.orc_extract_features.argtypes = [f32p, C.c_int64, C.c_int64, C.c_int32, C.c_float, C.c_int32,
                                       f32p, f32p, C.POINTER(C.c_int64)]
    L.orc_extract_features.restype = C.c_int64
    L.orc_sym3_eig.argtypes = [f64p, f64p]
    L.orc_edge_table.argtypes = [f32p, C.c_int64, C.c_float, C.c_float, f32p, i32p]
    L.orc_register_pair_edges.argtypes = [f32p, C.c_int64, f32p, C.c_int64, f32p, C.c_int64, f32p,
                                          C.c_int64, C.c_float, C.c_float, C.c_float, C.c_int32,
                                          C.c_int32, f64p, f64p, f64p, f64p, f64p,
                                          C.POINTER(C.c_int32), C.POINTER(C.c_int64)]
    L.orc_register_pair_edges.restype = C.c_int64
    L.orc_gmm_labels.argtypes = [f64p, C.c_int64, f64p, u8p, f64p, f64p]
    L.orc_gmm_labels.restype = C.c_int32
    L.orc_kabsch.argtypes = [f64p, f64p, C.c_int64, C.c_void_p, C.c_int32, f64p, f64p]
    L.orc_kabsch.restype = C.c_int32
    L.orc_quat_from_R.argtypes = [f64p, f64p]
    L.orc_quat_from_R.restype = C.c_int32
    L.orc_kabsch_f32.argtypes = [f32p, f32p, C.c_int64, C.c_void_p, C.c_int32, f64p, f64p, f64p]
    L.orc_kabsch_f32.restype = C.c_int32
    L.orc_svd3.argtypes = [f64p, f64p, f64p, f64p]
    L.orc_voxel_grid.argtypes = [f32p, C.c_int64, C.c_float, f32p]
    L.orc_voxel_grid.restype = C.c_int64
    L.orc_icp.argtypes = [f32p, C.c_int64, f32p, C.c_int64, C.POINTER(IcpParams), f32p,
                          C.POINTER(IcpResult)]
    L.orc_icp.restype = C.c_int32
    _lib = L
    return L


def profile(n_rows):
    p = Profile()
    if lib().orc_profile_get(n_rows, C.byref(p)) != 0:
        raise ValueError(f"unsupported N_SCAN_ROW {n_rows}")
    return p


# --------------------------------------------------------------------------- features
RING_CHAIN_FLOAT = 0     # std::atan(float) / std::sqrt(float) (libstdc++ <math.h>): the default
RING_CHAIN_DOUBLE = 1    # ::atan(double) / ::sqrt(double) only
RING_CHAINS = {"float": RING_CHAIN_FLOAT, "double": RING_CHAIN_DOUBLE}


class ring_chain:
    """with ring_chain("double"): every oracle ring id (bin_rings, extract_planes, ...) uses that
    evaluation of frameFeature.cpp:57, then the previous one again"""

    def __init__(self, chain):
        self.chain = RING_CHAINS[chain] if isinstance(chain, str) else int(chain)

    def __enter__(self):
        self.prev = lib().orc_set_ring_chain(self.chain)
        return self

    def __exit__(self, *exc):
        lib().orc_set_ring_chain(self.prev)
        return False


def ring_changes_f32(lo, hi, n_rows, cap=4096):
    """every change of the float chain's row id over ALL float ratios in [lo, hi] (exhaustive)
    -> (at [n] f32: the first float of each new id, id [n] i32)"""
    at = np.zeros(cap, np.float32)
    ids = np.zeros(cap, np.int32)
    n = lib().orc_ring_changes_f32(float(lo), float(hi), n_rows, at, ids, cap)
    assert n <= cap
    return at[:n], ids[:n]


def ring_ids(pts, n_rows):
    pts = np.ascontiguousarray(pts, np.float32)
    return np.array([lib().orc_ring_id(float(x), float(y), float(z), n_rows) for x, y, z in pts],
                    np.int32)


def bin_rings(pts, n_rows):
    """-> (rxyzi [kept,4] f32, ring_off [R+1] i64, src_idx [kept] i64, ring_of_input [n] i32)"""
    pts = np.ascontiguousarray(pts, np.float32)
    n = pts.shape[0]
    rx = np.zeros((max(n, 1), 4), np.float32)
    off = np.zeros(n_rows + 1, np.int64)
    src = np.zeros(max(n, 1), np.int64)
    rid = np.zeros(max(n, 1), np.int32)
    kept = lib().orc_bin(pts.reshape(-1), n, pts.shape[1], n_rows, rx.reshape(-1), off, src, rid)
    return rx[:kept], off, src[:kept], rid[:n]


def curvature(rxyzi, ring_off, n_rows):
    p = profile(n_rows)
    rx = np.ascontiguousarray(rxyzi, np.float32)
    cv = np.zeros(max(rx.shape[0], 1), np.float32)
    lib().orc_curvature(rx.reshape(-1) if rx.size else np.zeros(4, np.float32), ring_off, n_rows,
                        p.row_start, p.row_end, cv)
    return cv[:rx.shape[0]]


def select(rxyzi, curv, ring_off, n_rows):
    p = profile(n_rows)
    rx = np.ascontiguousarray(rxyzi, np.float32)
    n = rx.shape[0]
    out = np.zeros((max(n, 1), 4), np.float32)
    sel = np.zeros(max(n, 1), np.int64)
    m = lib().orc_select(rx.reshape(-1) if n else np.zeros(4, np.float32),
                         np.ascontiguousarray(curv, np.float32) if n else np.zeros(1, np.float32),
                         ring_off, n_rows, p.row_start, p.row_end, p.plane_min, p.plane_span,
                         out.reshape(-1), sel)
    return out[:m], sel[:m]


def extract_planes(pts, n_rows):
    """frameFeature cloudHandler: input xyz (n,3) -> plane cloud (m,4) x,y,z,intensity"""
    pts = np.ascontiguousarray(pts, np.float32)
    n = pts.shape[0]
    out = np.zeros((max(n, 1), 4), np.float32)
    m = lib().orc_extract_planes(pts.reshape(-1) if n else np.zeros(3, np.float32), n,
                                 pts.shape[1] if n else 3, n_rows, out.reshape(-1))
    if m < 0:
        raise ValueError("bad profile")
    return out[:m]


# --------------------------------------------------------------------------- registration
def ring_id_of_angle(angle, n_rows):
    return lib().orc_ring_id_of_angle(float(np.float32(angle)), n_rows)


def xknn(cloud, q, k):
    """k-NN through the oracle's x-sorted index (must equal knn())."""
    cloud = np.ascontiguousarray(cloud, np.float32)
    X = lib().orc_xindex_build(cloud.ctypes.data, cloud.shape[0])
    try:
        idx = np.zeros(k, np.int32)
        d2 = np.zeros(k, np.float32)
        qq = np.ascontiguousarray(q, np.float32)
        lib().orc_xindex_knn(X, qq.ctypes.data, k, idx.ctypes.data, d2.ctypes.data)
    finally:
        lib().orc_xindex_free(X)
    return idx, d2


def knn(cloud, q, k):
    cloud = np.ascontiguousarray(cloud, np.float32)
    idx = np.zeros(k, np.int32)
    d2 = np.zeros(k, np.float32)
    lib().orc_knn(cloud.reshape(-1), cloud.shape[0], np.ascontiguousarray(q, np.float32), k, idx, d2)
    return idx, d2


def plane_table(last, plane_max):
    last = np.ascontiguousarray(last, np.float32)
    m = last.shape[0]
    nrm = np.zeros((max(m, 1), 3), np.float32)
    valid = np.zeros(max(m, 1), np.int32)
    pick = np.zeros((max(m, 1), 5), np.int32)
    gate = np.zeros(max(m, 1), np.int32)
    if m:
        lib().orc_plane_table(last.reshape(-1), m, plane_max, nrm.reshape(-1), valid,
                              pick.reshape(-1), gate)
    return nrm[:m], valid[:m], pick[:m], gate[:m]


def transform_point(q, t, p):
    out = np.zeros(3, np.float32)
    lib().orc_transform_point(np.asarray(q, np.float64), np.asarray(t, np.float64),
                              np.ascontiguousarray(p, np.float32), out)
    return out


def correspond(last, curr, q, t):
    last = np.ascontiguousarray(last, np.float32)
    curr = np.ascontiguousarray(curr, np.float32)
    nn = np.zeros(max(curr.shape[0], 1), np.int32)
    lib().orc_correspond(last.reshape(-1), last.shape[0], curr.reshape(-1), curr.shape[0],
                         np.asarray(q, np.float64), np.asarray(t, np.float64), nn)
    return nn[:curr.shape[0]]


def solve(po, pa, nrm, mode=MODE_CERES_LM, max_iter=8, q_init=(0, 0, 0, 1), t_init=(0, 0, 0)):
    po = np.ascontiguousarray(po, np.float32).reshape(-1)
    pa = np.ascontiguousarray(pa, np.float32).reshape(-1)
    nr = np.ascontiguousarray(nrm, np.float32).reshape(-1)
    c = po.size // 3
    q = np.zeros(4); t = np.zeros(3)
    log = np.zeros(LOG_STRIDE * (max_iter + 2))
    nl = C.c_int32(0)
    lib().orc_solve(po if c else np.zeros(3, np.float32), pa if c else np.zeros(3, np.float32),
                    nr if c else np.zeros(3, np.float32), c, mode, max_iter,
                    np.asarray(q_init, np.float64), np.asarray(t_init, np.float64), q, t, log,
                    C.byref(nl))
    return q, t, log[:LOG_STRIDE * nl.value].reshape(-1, LOG_STRIDE)


def register_pair(last, curr, plane_max, mode=MODE_CERES_LM, max_iter=8, q_init=(0, 0, 0, 1),
                  t_init=(0, 0, 0)):
    """frameRegistration(): -> (q_xyzw, t, log [iters,10], n_corr)"""
    last = np.ascontiguousarray(last, np.float32)
    curr = np.ascontiguousarray(curr, np.float32)
    q = np.zeros(4); t = np.zeros(3)
    log = np.zeros(LOG_STRIDE * (max_iter + 2))
    nl = C.c_int32(0)
    c = lib().orc_register_pair(last.reshape(-1) if last.size else np.zeros(4, np.float32),
                                last.shape[0],
                                curr.reshape(-1) if curr.size else np.zeros(4, np.float32),
                                curr.shape[0], plane_max, mode, max_iter,
                                np.asarray(q_init, np.float64), np.asarray(t_init, np.float64),
                                q, t, log, C.byref(nl))
    return q, t, log[:LOG_STRIDE * nl.value].reshape(-1, LOG_STRIDE), c


# --------------------------------------------------------------------------- edges (beyond the
# reference; edge_oracle.c states the definitions -- parity unpinned)
EDGE_DEFAULTS = dict(edge_min=1.0, edge_span={64: 10, 16: 3}, line_ratio=3.0, max_nn_d2=1.0)


def _f32_or_dummy(a, width):
    a = np.ascontiguousarray(a, np.float32)
    return (a.reshape(-1) if a.size else np.zeros(width, np.float32)), (a.shape[0] if a.ndim else 0)


def select_edges(rxyzi, curv, ring_off, n_rows, edge_min=None, edge_span=None):
    p = profile(n_rows)
    edge_min = EDGE_DEFAULTS["edge_min"] if edge_min is None else edge_min
    edge_span = EDGE_DEFAULTS["edge_span"][n_rows] if edge_span is None else edge_span
    rx = np.ascontiguousarray(rxyzi, np.float32)
    n = rx.shape[0]
    out = np.zeros((max(n, 1), 4), np.float32)
    m = lib().orc_select_edges(rx.reshape(-1) if n else np.zeros(4, np.float32),
                               np.ascontiguousarray(curv, np.float32) if n else np.zeros(1, np.float32),
                               ring_off, n_rows, p.row_start, p.row_end, edge_min, edge_span,
                               out.reshape(-1))
    return out[:m]


def extract_features(pts, n_rows, edge_min=None, edge_span=None):
    """frameFeature with edges: -> (plane cloud (m,4), edge cloud (e,4))"""
    edge_min = EDGE_DEFAULTS["edge_min"] if edge_min is None else edge_min
    edge_span = EDGE_DEFAULTS["edge_span"][n_rows] if edge_span is None else edge_span
    pts = np.ascontiguousarray(pts, np.float32)
    n = pts.shape[0]
    planes = np.zeros((max(n, 1), 4), np.float32)
    edges = np.zeros((max(n, 1), 4), np.float32)
    me = C.c_int64(0)
    m = lib().orc_extract_features(pts.reshape(-1) if n else np.zeros(3, np.float32), n,
                                   pts.shape[1] if n else 3, n_rows, edge_min, edge_span,
                                   planes.reshape(-1), edges.reshape(-1), C.byref(me))
    if m < 0:
        raise ValueError("bad profile")
    return planes[:m], edges[:me.value]


def sym3_eig(A):
    A = np.array(A, np.float64).reshape(9).copy()
    V = np.zeros(9)
    lib().orc_sym3_eig(A, V)
    return A.reshape(3, 3).diagonal().copy(), V.reshape(3, 3)


def edge_table(edges, max_nn_d2=None, line_ratio=None):
    """-> (line [m,6] f32: centroid, direction; valid [m] i32)"""
    max_nn_d2 = EDGE_DEFAULTS["max_nn_d2"] if max_nn_d2 is None else max_nn_d2
    line_ratio = EDGE_DEFAULTS["line_ratio"] if line_ratio is None else line_ratio
    e, m = _f32_or_dummy(edges, 4)
    line = np.zeros((max(m, 1), 6), np.float32)
    valid = np.zeros(max(m, 1), np.int32)
    if m:
        lib().orc_edge_table(e, m, max_nn_d2, line_ratio, line.reshape(-1), valid)
    return line[:m], valid[:m]


def register_pair_edges(last, curr, last_e, curr_e, plane_max, mode=MODE_CERES_LM, max_iter=8,
                        q_init=(0, 0, 0, 1), t_init=(0, 0, 0), max_nn_d2=None, line_ratio=None):
    """frameRegistration with point-to-plane AND point-to-line blocks:
    -> (q_xyzw, t, log [iters,10], n_plane_corr, n_edge_corr)"""
    max_nn_d2 = EDGE_DEFAULTS["max_nn_d2"] if max_nn_d2 is None else max_nn_d2
    line_ratio = EDGE_DEFAULTS["line_ratio"] if line_ratio is None else line_ratio
    L, ml = _f32_or_dummy(last, 4)
    Cc, mc = _f32_or_dummy(curr, 4)
    Le, mle = _f32_or_dummy(last_e, 4)
    Ce, mce = _f32_or_dummy(curr_e, 4)
    q = np.zeros(4); t = np.zeros(3)
    log = np.zeros(LOG_STRIDE * (max_iter + 2))
    nl = C.c_int32(0)
    ne = C.c_int64(0)
    c = lib().orc_register_pair_edges(L, ml, Cc, mc, Le, mle, Ce, mce, plane_max, max_nn_d2,
                                      line_ratio, mode, max_iter, np.asarray(q_init, np.float64),
                                      np.asarray(t_init, np.float64), q, t, log, C.byref(nl),
                                      C.byref(ne))
    return q, t, log[:LOG_STRIDE * nl.value].reshape(-1, LOG_STRIDE), c, ne.value


def accumulate(q0l, t0l, qlc, tlc):
    q = np.zeros(4); t = np.zeros(3)
    lib().orc_accumulate(*(np.asarray(v, np.float64) for v in (q0l, t0l, qlc, tlc)), q, t)
    return q, t


# --------------------------------------------------------------------------- mask + Kabsch
class LegacyRandomState:
    """numpy RandomState (MT19937) restated in C: random_sample() stream."""

    def __init__(self, seed):
        class MT(C.Structure):
            _fields_ = [("mt", C.c_uint32 * 624), ("pos", C.c_int32)]
        self._st = MT()
        L = lib()
        L.orc_mt_seed.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_mt_random_sample.argtypes = [C.c_void_p]
        L.orc_mt_random_sample.restype = C.c_double
        L.orc_mt_seed(C.byref(self._st), seed)

    def random_sample(self, n=None):
        L = lib()
        if n is None:
            return L.orc_mt_random_sample(C.byref(self._st))
        return np.array([L.orc_mt_random_sample(C.byref(self._st)) for _ in range(n)])


def gmm_labels(X, draws):
    """GaussianMixture(2).fit_predict restated -> (labels u8, info dict, means [2,6])"""
    X = np.ascontiguousarray(X, np.float64)
    n = X.shape[0]
    lab = np.zeros(n, np.uint8)
    info = np.zeros(8)
    means = np.zeros(12)
    rc = lib().orc_gmm_labels(X.reshape(-1), n, np.asarray(draws, np.float64), lab, info, means)
    if rc != 0:
        raise ValueError(f"oracle gmm failed rc={rc}")
    keys = ["kmeans_iter", "em_iter", "converged", "center0", "center1", "bg_label", "n_bg",
            "lower_bound"]
    d = dict(zip(keys, info.tolist()))
    return lab, d, means.reshape(2, 6)


def kabsch(src, dst, mask=None, reflection=0):
    src = np.ascontiguousarray(src, np.float64)
    dst = np.ascontiguousarray(dst, np.float64)
    R = np.zeros(9); t = np.zeros(3)
    m = None
    if mask is not None:
        m = np.ascontiguousarray(mask, np.uint8)
    rc = lib().orc_kabsch(src.reshape(-1), dst.reshape(-1), src.shape[0],
                          m.ctypes.data if m is not None else None, reflection, R, t)
    return rc, R.reshape(3, 3), t


def quat_from_R(R):
    q = np.zeros(4)
    rc = lib().orc_quat_from_R(np.ascontiguousarray(R, np.float64).reshape(-1), q)
    return rc, q


def svd3(A):
    U = np.zeros(9); S = np.zeros(3); Vt = np.zeros(9)
    lib().orc_svd3(np.ascontiguousarray(A, np.float64).reshape(-1), U, S, Vt)
    return U.reshape(3, 3), S, Vt.reshape(3, 3)


def kabsch_f32(pos, flow, mask=None, reflection=0):
    """slove_RT_by_SVD(points[bg] + flow[bg], points[bg]) + Quaternion on float32 arrays, as the
    ASF block runs it (main_sju_occ_ros.py:273-284, :455-473); see orc_kabsch_f32.
    -> rc, R (3, 3) f32 values, t (3,) f32 values, q_xyzw (4,)"""
    pos = np.ascontiguousarray(pos, np.float32)
    flow = np.ascontiguousarray(flow, np.float32)
    R = np.zeros(9); t = np.zeros(3); q = np.zeros(4)
    m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    rc = lib().orc_kabsch_f32(pos.reshape(-1), flow.reshape(-1), pos.shape[0],
                              m.ctypes.data if m is not None else None, reflection, R, t, q)
    return rc, R.reshape(3, 3), t, q


def mask_and_pose(points, flow, draws, kabsch_dtype="float64"):
    """PointCloudOdometry_noSeg.py:97-125 restated: GMM mask, Kabsch(points+flow, points),
    quaternion.  kabsch_dtype "float32": the Kabsch + quaternion tail on float32 arrays, as the
    ASF block runs it on float32 network flow (kabsch_f32).
    -> dict(labels, bg_mask, R, t, q_xyzw, info, rc)"""
    X = np.concatenate([np.asarray(flow, np.float64), np.asarray(points, np.float64)], axis=1)
    lab, info, means = gmm_labels(X, draws)
    bg = (lab == int(info["bg_label"])).astype(np.uint8)
    if kabsch_dtype == "float32":
        rc, R, t, q = kabsch_f32(points, flow, bg)
        return dict(labels=lab, bg_mask=bg, R=R, t=t, q_xyzw=q, info=info, means=means, rc=rc)
    p = np.asarray(points, np.float64)
    rc, R, t = kabsch(p + np.asarray(flow, np.float64), p, bg)
    qrc, q = quat_from_R(R) if rc == 0 else (rc, np.zeros(4))
    return dict(labels=lab, bg_mask=bg, R=R, t=t, q_xyzw=q, info=info, means=means,
                rc=rc if rc != 0 else qrc)


# ---- mapOptmization loop closure: oracle/loop_oracle.c ----
def voxel_grid(xyzi, leaf):
    """pcl::VoxelGrid<PointXYZI> restated (mapOptmization.cpp:214-217): n x 4 -> m x 4."""
    x = np.ascontiguousarray(xyzi, np.float32).reshape(-1, 4)
    out = np.zeros_like(x)
    m = lib().orc_voxel_grid(x.reshape(-1), x.shape[0], float(leaf), out.reshape(-1))
    return out[:m].copy()


def icp(src, tgt, max_corr_dist=50.0, max_iter=100, trans_eps=1e-6, fit_eps=1e-6, guess=None):
    """pcl::IterativeClosestPoint<PointXYZI, PointXYZI> restated (mapOptmization.cpp:224-236)."""
    s = np.ascontiguousarray(src, np.float32).reshape(-1, 4)
    t = np.ascontiguousarray(tgt, np.float32).reshape(-1, 4)
    g = np.eye(4, dtype=np.float32) if guess is None else np.ascontiguousarray(guess, np.float32)
    p = IcpParams(int(max_iter), float(max_corr_dist), float(trans_eps), float(fit_eps))
    r = IcpResult()
    lib().orc_icp(s.reshape(-1), s.shape[0], t.reshape(-1), t.shape[0], C.byref(p), g.reshape(-1),
                  C.byref(r))
    return dict(T=np.array(r.T, np.float32).reshape(4, 4), fitness=r.fitness,
                converged=bool(r.converged), iterations=r.iterations,
                state=ICP_STATES[r.state], n_corr=r.n_corr)


# ---- TFlow point-set operators: oracle/pn2_oracle.c ----
def _pn2(L):
    if not getattr(L, "_pn2_typed", False):
        L.orc_pn2_fps.argtypes = [f32p, C.c_int64, C.c_int32, C.c_int32, f32p, i32p]
        L.orc_pn2_knn.argtypes = [f32p, C.c_int64, f32p, C.c_int64, C.c_int32, f32p, i32p]
        L.orc_pn2_gather.argtypes = [f32p, C.c_int32, C.c_int64, i32p, C.c_int64, f32p]
        L.orc_pn2_interp3.argtypes = [f32p, C.c_int32, C.c_int64, i32p, f32p, C.c_int64, f32p]
        L.orc_pn2_upsample.argtypes = [f32p, C.c_int64, f32p, C.c_int64, f32p, C.c_int32,
                                       C.c_int32, f32p]
        L._pn2_typed = True
    return L


def pn2_fps(xyz, npoint, start=None):
    """farthest_point_sample (utils/utils.py:68-89): xyz [B, N, 3] -> int32 [B, npoint]."""
    L = _pn2(lib())
    x = np.ascontiguousarray(xyz, np.float32)
    B, N, _ = x.shape
    out = np.zeros((B, npoint), np.int32)
    tmp = np.zeros(N, np.float32)
    for b in range(B):
        o = np.zeros(npoint, np.int32)
        L.orc_pn2_fps(np.ascontiguousarray(x[b]).reshape(-1), N, npoint,
                      0 if start is None else int(start[b]), tmp, o)
        out[b] = o
    return out


def pn2_knn(k, query, ref):
    """knn_point (utils/utils.py:92-108): query [B, S, 3], ref [B, N, 3] -> (dist, idx) [B, S, k]."""
    L = _pn2(lib())
    q = np.ascontiguousarray(query, np.float32)
    r = np.ascontiguousarray(ref, np.float32)
    B, S, _ = q.shape
    N = r.shape[1]
    dist = np.zeros((B, S, k), np.float32)
    idx = np.zeros((B, S, k), np.int32)
    for b in range(B):
        d = np.zeros(S * k, np.float32); i = np.zeros(S * k, np.int32)
        L.orc_pn2_knn(np.ascontiguousarray(q[b]).reshape(-1), S,
                      np.ascontiguousarray(r[b]).reshape(-1), N, k, d, i)
        dist[b] = d.reshape(S, k); idx[b] = i.reshape(S, k)
    return dist, idx


def pn2_gather(feat, idx):
    """index_points on the [B, C, N] layout: idx [B, ...] -> [B, C, ...]."""
    L = _pn2(lib())
    f = np.ascontiguousarray(feat, np.float32)
    ix = np.ascontiguousarray(idx, np.int32)
    B, Cc, N = f.shape
    g = int(np.prod(ix.shape[1:]))
    out = np.zeros((B, Cc, g), np.float32)
    for b in range(B):
        o = np.zeros(Cc * g, np.float32)
        L.orc_pn2_gather(np.ascontiguousarray(f[b]).reshape(-1), Cc, N,
                         np.ascontiguousarray(ix[b]).reshape(-1), g, o)
        out[b] = o.reshape(Cc, g)
    return out.reshape((B, Cc) + ix.shape[1:])


def pn2_three_interpolate(feat, idx, weight):
    """utils/utils.py:662-663: feat [B, C, M], idx/weight [B, N, 3] -> [B, C, N]."""
    L = _pn2(lib())
    f = np.ascontiguousarray(feat, np.float32)
    ix = np.ascontiguousarray(idx, np.int32)
    w = np.ascontiguousarray(weight, np.float32)
    B, Cc, M = f.shape
    N = ix.shape[1]
    out = np.zeros((B, Cc, N), np.float32)
    for b in range(B):
        o = np.zeros(Cc * N, np.float32)
        L.orc_pn2_interp3(np.ascontiguousarray(f[b]).reshape(-1), Cc, M,
                          np.ascontiguousarray(ix[b]).reshape(-1),
                          np.ascontiguousarray(w[b]).reshape(-1), N, o)
        out[b] = o.reshape(Cc, N)
    return out


def pn2_upsample_flow(xyz, sparse_xyz, sparse_feat, k=3):
    """UpsampleFlow.forward (utils/soflow.py:1442-1470): xyz [B, 3, N], sparse_xyz [B, 3, S],
    sparse_feat [B, C, S] -> [B, C, N]."""
    L = _pn2(lib())
    x = np.ascontiguousarray(xyz, np.float32)
    sx = np.ascontiguousarray(sparse_xyz, np.float32)
    sf = np.ascontiguousarray(sparse_feat, np.float32)
    B, _, N = x.shape
    S = sx.shape[2]
    Cc = sf.shape[1]
    out = np.zeros((B, Cc, N), np.float32)
    for b in range(B):
        o = np.zeros(Cc * N, np.float32)
        L.orc_pn2_upsample(np.ascontiguousarray(x[b]).reshape(-1), N,
                           np.ascontiguousarray(sx[b]).reshape(-1), S,
                           np.ascontiguousarray(sf[b]).reshape(-1), Cc, int(k), o)
        out[b] = o.reshape(Cc, N)
    return out
