"""ctypes binding of libssf_frontend.so (include/ssf_frontend.h).

The library is loaded AFTER torch so that its libamdhip64.so.7 dependency resolves to the HIP
runtime torch already mapped (one runtime per process).  There is no fallback: if the library
is missing or fails to load, every entry point raises -- the product path never silently runs
on a CPU substitute.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede the dlopen below, see module docstring)

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
LIB_PATH = os.environ.get("SSF_LIB", os.path.join(LIB_DIR, "libssf_frontend.so"))

SSF_OK, SSF_E_ARG, SSF_E_HIP, SSF_E_NOMEM, SSF_E_CAPACITY, SSF_E_NODEV = 0, -1, -2, -3, -4, -5
SOLVER_CERES_LM, SOLVER_GN = 0, 1
MASK_GMM, MASK_GT, MASK_GIVEN = 0, 1, 2
# the evaluation of frameFeature.cpp:57 (ssf_config.ring_chain, include/ssf_frontend.h)
RING_CHAIN_FLOAT, RING_CHAIN_DOUBLE = 0, 1
RING_CHAINS = {"float": RING_CHAIN_FLOAT, "double": RING_CHAIN_DOUBLE}
# frames of plane points the association can stage from the plane table's strip image
# (registration.hip: kStripHeadWords, kAssocStripF4Max)
STRIP_IMAGE_MIN, STRIP_IMAGE_MAX = (256 + 1) + 2 * 256 + 4, 6144
POSE_OUT_STRIDE = 32
POSE_OUT = dict(T=0, Q=3, R=7, STATUS=16, NBG=17, BGLABEL=18, KM_ITER=19, EM_ITER=20,
                CONVERGED=21, CENTER0=22, CENTER1=23, LOWER_BOUND=24, PASSES=25)
POSE_EMPTY, POSE_REFLECTION, POSE_NOT_ORTHOGONAL, POSE_GMM_FAILED, POSE_SYNC_FAILED = -1, -2, -3, -4, -5

# Every symbol include/ssf_frontend.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "ssf_abi_version", "ssf_config_default", "ssf_create", "ssf_destroy", "ssf_last_error",
    "ssf_reserve", "ssf_extract_planes_batch", "ssf_extract_planes", "ssf_plane_table_batch",
    "ssf_register_batch", "ssf_register_chain", "ssf_mask_pose_batch", "ssf_rng_seed", "ssf_accumulate_sequence",
    "ssf_voxel_grid_batch", "ssf_icp_params_default", "ssf_icp_batch",
    "ssf_extract_planes_batch_masked", "ssf_register_pair", "ssf_profile_enable",
    "ssf_profile_read", "ssf_set_mask_split", "ssf_mask_pose_batch_f64",
    "ssf_edge_config_default", "ssf_set_edge_config", "ssf_extract_features_batch",
    "ssf_edge_table_batch", "ssf_register_batch_edges", "ssf_kabsch_f32_batch",
    "ssf_set_mask_schedule",
]
# Every symbol include/ssf_pointnet2.h declares (TFlow point-set operators).
PN2_EXPORTS = [
    "ssf_pn2_last_error", "ssf_pn2_furthest_point_sample", "ssf_pn2_knn", "ssf_pn2_three_nn",
    "ssf_pn2_gather", "ssf_pn2_three_interpolate", "ssf_pn2_upsample_flow",
    "ssf_pn2_group_relative",
]
PN2_KNN_MAX, PN2_UPSAMPLE_MAX_SPARSE = 32, 4096

ICP_OUT_STRIDE = 24
ICP_OUT = dict(T=0, FITNESS=16, CONVERGED=17, ITERATIONS=18, STATE=19, NCORR=20)
ICP_STATES = {0: "not_converged", 1: "iterations", 2: "transform", 3: "abs_mse", 4: "rel_mse",
              5: "no_correspondences"}


class IcpParams(C.Structure):
    _fields_ = [("max_iter", C.c_int32), ("max_corr_dist", C.c_float), ("trans_eps", C.c_double),
                ("fit_eps", C.c_double)]


STEP_STATUS = {0: "rejected", 1: "accepted", 2: "invalid", 3: "param_tol", 4: "func_tol",
               5: "grad_tol", 6: "gn"}


class Step(C.Structure):
    _fields_ = [("q", C.c_double * 4), ("t", C.c_double * 3), ("cost", C.c_double),
                ("status", C.c_int32), ("pad", C.c_int32), ("radius", C.c_double)]


class StepLog(C.Structure):
    _fields_ = [("cap", C.c_int32), ("n_steps", C.c_int32), ("n_corr", C.c_int32),
                ("pad", C.c_int32), ("steps", C.POINTER(Step))]


class KernelTime(C.Structure):
    _fields_ = [("name", C.c_char * 48), ("launches", C.c_int32), ("total_ms", C.c_double)]


class Config(C.Structure):
    _fields_ = [("n_rows", C.c_int32), ("plane_min", C.c_float), ("plane_span", C.c_int32),
                ("row_start", C.c_int32), ("row_end", C.c_int32), ("plane_max", C.c_float),
                ("solver", C.c_int32), ("max_iter", C.c_int32), ("ring_chain", C.c_int32)]


class EdgeConfig(C.Structure):
    """ssf_edge_config (beyond the reference: edge features + point-to-line residuals)."""
    _fields_ = [("edge_min", C.c_float), ("edge_span", C.c_int32), ("line_ratio", C.c_float),
                ("max_nn_d2", C.c_float)]


_lib = None


class SSFError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SSFError(f"{LIB_PATH} is missing: build it first (python -c 'import __graft_entry__ "
                       f"as g; g.build()')")
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, dbl = C.c_void_p, C.c_int32, C.c_int64, C.c_double
    L.ssf_abi_version.restype = i32
    L.ssf_config_default.argtypes = [i32, C.POINTER(Config)]
    L.ssf_config_default.restype = i32
    L.ssf_create.argtypes = [i32, C.POINTER(Config), C.POINTER(vp)]
    L.ssf_create.restype = i32
    L.ssf_destroy.argtypes = [vp]
    L.ssf_destroy.restype = None
    L.ssf_last_error.argtypes = [vp]
    L.ssf_last_error.restype = C.c_char_p
    L.ssf_reserve.argtypes = [vp, i32, i64]
    L.ssf_reserve.restype = i32
    L.ssf_rng_seed.argtypes = [vp, C.c_uint32]
    L.ssf_rng_seed.restype = i32
    L.ssf_extract_planes_batch.argtypes = [vp, vp, i32, vp, i32, vp, i64, i64, vp, vp, vp, vp, vp]
    L.ssf_extract_planes_batch.restype = i32
    L.ssf_extract_planes_batch_masked.argtypes = [vp, vp, i32, vp, i32, vp, i64, i64, vp, vp, vp, vp, vp, vp]
    L.ssf_extract_planes_batch_masked.restype = i32
    L.ssf_extract_planes.argtypes = [vp, vp, vp, i64, i32, i32, vp, C.POINTER(i64), i64]
    L.ssf_extract_planes.restype = i32
    L.ssf_plane_table_batch.argtypes = [vp, vp, i32, vp, vp, vp, i64, vp, vp, vp, vp, vp, vp]
    L.ssf_plane_table_batch.restype = i32
    L.ssf_register_batch.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64,
                                     vp, vp, vp, vp, vp, vp, vp, vp]
    L.ssf_register_batch.restype = i32
    L.ssf_register_chain.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, vp, vp, i64, i64,
                                     vp, vp, vp, vp, vp, vp, vp]
    L.ssf_register_chain.restype = i32
    L.ssf_register_pair.argtypes = [vp, vp, vp, i64, vp, i64, vp, vp, vp, vp, C.POINTER(StepLog)]
    L.ssf_register_pair.restype = i32
    L.ssf_set_mask_split.argtypes = [vp, i32]
    L.ssf_set_mask_split.restype = i32
    L.ssf_set_mask_schedule.argtypes = [vp, vp, i32, i32]
    L.ssf_set_mask_schedule.restype = i32
    L.ssf_profile_enable.argtypes = [vp, i32]
    L.ssf_profile_enable.restype = i32
    L.ssf_profile_read.argtypes = [vp, C.POINTER(KernelTime), i32, C.POINTER(i32)]
    L.ssf_profile_read.restype = i32
    L.ssf_mask_pose_batch.argtypes = [vp, vp, i32, vp, vp, vp, vp, i32, vp, vp, i32, vp, vp]
    L.ssf_mask_pose_batch.restype = i32
    L.ssf_mask_pose_batch_f64.argtypes = [vp, vp, i32, vp, vp, vp, vp, i32, vp, vp, i32, vp, vp]
    L.ssf_mask_pose_batch_f64.restype = i32
    L.ssf_kabsch_f32_batch.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, i32, i32, vp]
    L.ssf_kabsch_f32_batch.restype = i32
    L.ssf_edge_config_default.argtypes = [i32, C.POINTER(EdgeConfig)]
    L.ssf_edge_config_default.restype = i32
    L.ssf_set_edge_config.argtypes = [vp, C.POINTER(EdgeConfig)]
    L.ssf_set_edge_config.restype = i32
    L.ssf_extract_features_batch.argtypes = [vp, vp, i32, vp, i32, vp, i64, i64, vp, vp, vp, vp, vp]
    L.ssf_extract_features_batch.restype = i32
    L.ssf_edge_table_batch.argtypes = [vp, vp, i32, vp, vp, vp, i64, vp, vp]
    L.ssf_edge_table_batch.restype = i32
    L.ssf_register_batch_edges.argtypes = ([vp, vp, i32] + [vp] * 10 + [i64, i64] + [vp] * 8 +
                                           [i64, i64] + [vp] * 8)
    L.ssf_register_batch_edges.restype = i32
    L.ssf_accumulate_sequence.argtypes = [vp, vp, i32, vp, vp, vp]
    L.ssf_accumulate_sequence.restype = i32
    L.ssf_voxel_grid_batch.argtypes = [vp, vp, i32, vp, vp, vp, C.c_float, vp, vp]
    L.ssf_voxel_grid_batch.restype = i32
    L.ssf_icp_params_default.argtypes = [C.POINTER(IcpParams)]
    L.ssf_icp_params_default.restype = i32
    L.ssf_icp_batch.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, vp, C.POINTER(IcpParams), vp, vp]
    L.ssf_icp_batch.restype = i32
    L.ssf_pn2_last_error.argtypes = []
    L.ssf_pn2_last_error.restype = C.c_char_p
    L.ssf_pn2_furthest_point_sample.argtypes = [vp, i32, i32, i32, vp, vp, vp, vp]
    L.ssf_pn2_knn.argtypes = [vp, i32, i32, i32, i32, vp, vp, vp, vp]
    L.ssf_pn2_three_nn.argtypes = [vp, i32, i32, i32, vp, vp, vp, vp]
    L.ssf_pn2_gather.argtypes = [vp, i32, i32, i32, i32, vp, vp, vp, vp]
    L.ssf_pn2_three_interpolate.argtypes = [vp, i32, i32, i32, i32, vp, vp, vp, vp, vp]
    L.ssf_pn2_upsample_flow.argtypes = [vp, i32, i32, i32, i32, i32, vp, vp, vp, vp]
    L.ssf_pn2_group_relative.argtypes = [vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp]
    for name in PN2_EXPORTS[1:]:
        getattr(L, name).restype = i32
    _lib = L
    return L


def config_default(n_rows: int) -> Config:
    cfg = Config()
    if lib().ssf_config_default(n_rows, C.byref(cfg)) != SSF_OK:
        raise ValueError(f"unsupported N_SCAN_ROW {n_rows} (16 or 64)")
    return cfg
