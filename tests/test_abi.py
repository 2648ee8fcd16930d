"""CPU-side checks of the C-ABI boundary: the library loads, exports every symbol declared in
include/ssf_frontend.h, and the host-only entry points behave (no GPU compute is called)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ssf_frontend.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ssf_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from ssf import _abi
    L = _abi.lib()
    syms = declared_symbols()
    assert len(syms) >= 13
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(_abi.EXPORTS) == syms


def test_abi_version_and_profiles():
    from ssf import _abi
    L = _abi.lib()
    assert L.ssf_abi_version() == 2
    c64 = _abi.config_default(64)
    assert (c64.n_rows, c64.plane_span, c64.row_start, c64.row_end, c64.max_iter) == (64, 25, 5, 5, 8)
    assert c64.ring_chain == _abi.RING_CHAIN_FLOAT         # frameFeature.cpp:57 under libstdc++
    assert c64.plane_min == np.float32(0.005) and c64.plane_max == np.float32(0.05)
    c16 = _abi.config_default(16)
    assert (c16.plane_span, c16.row_start, c16.row_end) == (3, 0, 0)
    assert c16.plane_min == np.float32(0.05) and c16.plane_max == np.float32(0.15)
    with pytest.raises(ValueError):
        _abi.config_default(32)


def test_error_paths_without_gpu():
    """null context / bad args are rejected before any HIP call"""
    from ssf import _abi
    L = _abi.lib()
    assert L.ssf_reserve(None, 1, 1) == _abi.SSF_E_ARG
    assert L.ssf_rng_seed(None, 1) == _abi.SSF_E_ARG
    assert L.ssf_extract_planes_batch(None, None, 1, None, 3, None, 0, 0, None, None, None, None, None) == _abi.SSF_E_ARG
    assert L.ssf_last_error(None) == b"null context"
    assert L.ssf_register_chain(None, None, 1, *([None] * 7), 0, 0, *([None] * 7)) == _abi.SSF_E_ARG
    assert L.ssf_voxel_grid_batch(None, None, 1, None, None, None, 0.1, None, None) == _abi.SSF_E_ARG
    prm = _abi.IcpParams()
    assert L.ssf_icp_params_default(C.byref(prm)) == _abi.SSF_OK
    assert (prm.max_iter, prm.max_corr_dist, prm.trans_eps, prm.fit_eps) == (100, 50.0, 1e-6, 1e-6)
    assert L.ssf_icp_params_default(None) == _abi.SSF_E_ARG
    assert L.ssf_icp_batch(None, None, 1, None, None, None, None, None, None, C.byref(prm), None, None) == _abi.SSF_E_ARG
    cfg = _abi.config_default(64)
    cfg.n_rows = 33
    h = C.c_void_p()
    assert L.ssf_create(0, C.byref(cfg), C.byref(h)) == _abi.SSF_E_ARG


def test_no_cpu_fallback_in_product_package():
    """the product package never imports the oracle"""
    pkg = os.path.join(REPO, "ssf-slam_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".cpp", ".h")):
                txt = open(os.path.join(root, f)).read()
                # citations of the oracle's C files in comments are documentation, not a link
                txt = re.sub(r"oracle/\w+\.c", "", txt)
                assert "oracle" not in txt.replace("CPU oracle", "").replace("the oracle", "") or f == "synth.py", f


def test_pointnet2_header_symbols_exported_and_arg_checks():
    """include/ssf_pointnet2.h: every declared symbol is exported; bad arguments are rejected
    before any HIP call"""
    from ssf import _abi
    L = _abi.lib()
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(REPO, "include", "ssf_pointnet2.h")).read(), flags=re.S)
    syms = sorted(set(re.findall(r"\b(ssf_[a-z0-9_]+)\s*\(", src)))
    assert syms == sorted(_abi.PN2_EXPORTS)
    assert all(hasattr(L, s) for s in syms)
    assert L.ssf_pn2_knn(None, 1, 4, 8, 33, 1, 1, 1, 1) == _abi.SSF_E_ARG      # k > 32
    assert b"knn" in L.ssf_pn2_last_error()
    assert L.ssf_pn2_furthest_point_sample(None, 1, 0, 4, 1, None, None, 1) == _abi.SSF_E_ARG
    assert L.ssf_pn2_furthest_point_sample(None, 1, 20000, 4, 1, None, None, 1) == _abi.SSF_E_ARG  # no temp
    assert L.ssf_pn2_upsample_flow(None, 1, 8, 5000, 3, 3, 1, 1, 1, 1) == _abi.SSF_E_ARG  # s > 4096
    assert L.ssf_pn2_gather(None, 1, 1, 4, 4, 1, 1, 1, None) == _abi.SSF_E_ARG
    assert L.ssf_pn2_group_relative(None, 1, 40000, 4, 4, 0, 1, 1, None, 1, 1, 1) == _abi.SSF_E_ARG  # n too big


def test_pointnet2_python_mirror_rejects_host_tensors():
    """ssf.pointnet2 has no CPU path: host tensors are refused before any library call"""
    import torch
    from ssf import pointnet2 as P
    x = torch.zeros(1, 8, 3)
    for call in (lambda: P.furthest_point_sample(x, 4), lambda: P.knn(3, x, x),
                 lambda: P.three_nn(x, x), lambda: P.gather_operation(torch.zeros(1, 2, 8), torch.zeros(1, 4)),
                 lambda: P.upsample_flow(torch.zeros(1, 3, 8), torch.zeros(1, 3, 4), torch.zeros(1, 3, 4))):
        with pytest.raises(ValueError, match="CUDA"):
            call()
