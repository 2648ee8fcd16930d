"""examples/frame_registration.cpp: the INTEGRATION.md C-ABI bindings (cloudHandler() ->
ssf_extract_planes, frameRegistration() -> ssf_register_pair) compiled as a plain g++ host
program.  CPU: it compiles against include/ and the in-tree library, and refuses cleanly without
a device.  GPU: its pose equals the Python host's and the oracle's on the same two scans."""
import json
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "examples", "frame_registration.cpp")
LIBDIR = os.path.join(REPO, "ssf-slam_amd", "ssf", "_lib")
EXE = os.path.join(REPO, "examples", "_bin", "frame_registration")


def _compile(out):
    return subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"),
                           "-I", "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", SRC, "-L", LIBDIR,
                           "-lssf_frontend", "-L", "/opt/rocm/lib", "-lamdhip64",
                           f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath,/opt/rocm/lib", "-o", out],
                          capture_output=True, text=True, timeout=300)


def test_example_compiles_and_refuses_without_device(tmp_path):
    if not os.path.exists(os.path.join(LIBDIR, "libssf_frontend.so")):
        pytest.skip("library not built")
    exe = str(tmp_path / "frame_registration")
    r = _compile(exe)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr
    a = tmp_path / "a.bin"
    np.zeros((100, 3), np.float32).tofile(a)
    r = subprocess.run([exe, str(a), str(a)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, HIP_VISIBLE_DEVICES="-1"))
    assert r.returncode == 1 and "ssf_create failed" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["lm", "gn"])
def test_example_pose_matches_python_and_oracle(oracle, dev, tmp_path, mode):
    import torch
    import ssf
    from ssf import synth
    assert os.access(EXE, os.X_OK), "examples/_bin/frame_registration not built (build())"
    sc = synth.Scene(5)
    clouds = [synth.scan(5, k, n_az=900, scene=sc)["pos1"].numpy() for k in range(2)]
    paths = []
    for k, c in enumerate(clouds):
        p = tmp_path / f"f{k}.bin"
        np.ascontiguousarray(c, np.float32).tofile(p)
        paths.append(str(p))
    r = subprocess.run([EXE, *paths] + (["gn"] if mode == "gn" else []), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout)
    solver, iters, omode = ("gn", 10, oracle.MODE_GN) if mode == "gn" else ("ceres_lm", 8, oracle.MODE_CERES_LM)
    fe = ssf.Frontend(64, device=dev.index, solver=solver, max_iter=iters)
    planes = [oracle.extract_planes(c, 64) for c in clouds]
    assert [got["m_last"], got["m_curr"]] == [len(p) for p in planes]
    q, t, steps, nc = fe.register_pair(torch.from_numpy(planes[0]).to(dev), torch.from_numpy(planes[1]).to(dev))
    assert got["n_corr"] == nc and len(got["steps"]) == len(steps)
    assert np.abs(np.array(got["q"]) - q).max() < 1e-12 and np.abs(np.array(got["t"]) - t).max() < 1e-12
    qr, tr, _, cr = oracle.register_pair(planes[0], planes[1], 0.05, mode=omode, max_iter=iters)
    assert nc == cr
    assert np.abs(np.array(got["t"]) - tr).max() < 1e-5
    d = abs(float(np.dot(np.array(got["q"]), qr)))
    assert 2.0 * np.arcsin(min(1.0, np.sqrt(max(0.0, 1.0 - d * d)))) < 1e-6
