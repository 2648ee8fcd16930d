"""Build libssf_frontend.so for gfx950 with hipcc (no cmake, no JIT cache: the .so is written
in-tree under ssf/_lib/ so it travels with the repository snapshot to the GPU box)."""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "ssf", "_lib")
OBJ_DIR = os.path.join(HERE, "build")
LIB = os.path.join(OUT_DIR, "libssf_frontend.so")
SYNTH_LIB = os.path.join(OUT_DIR, "libssf_synth.so")
SOURCES = ["abi.hip", "features.hip", "registration.hip", "mask_pose.hip", "mask_pose_f64.hip", "kabsch_f32.hip",
           "loop.hip", "pointnet2.hip"]
# sources that include another source file
SRC_DEPS = {"mask_pose_f64.hip": ["mask_pose.hip"]}
HEADERS = ["ssf_device.hpp", "ssf_internal.hpp", "svd3.hpp", os.path.join("..", "..", "include", "ssf_frontend.h"),
           os.path.join("..", "..", "include", "ssf_pointnet2.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -ffp-contract=off: no FMA contraction, so float stages match the reference's x86 arithmetic
# (and the CPU oracle) bit for bit.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-Wall"]
# The f64 GMM/Kabsch kernel is compared with tolerances (labels, iteration counts, 1e-5 m), not
# bit for bit, so it may contract multiply-adds into FMAs (half the f64 instructions).
FILE_FLAGS = {"mask_pose.hip": ["-ffp-contract=fast"], "mask_pose_f64.hip": ["-ffp-contract=fast"]}


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OUT_DIR, exist_ok=True)
    os.makedirs(OBJ_DIR, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS]
    objs, jobs = [], []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ_DIR, src.replace(".hip", ".o"))
        objs.append(o)
        if force or _stale(o, [s] + hdrs + [os.path.join(CSRC, d) for d in SRC_DEPS.get(src, [])]):
            jobs.append([HIPCC, *FLAGS, *FILE_FLAGS.get(src, []), "-c", s, "-o", o])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r

    with ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    if force or jobs or _stale(LIB, objs):
        run([HIPCC, *FLAGS, "-shared", *objs, "-o", LIB])
    # bench / test data generator (ssf.synth.BatchScanner): a library of its own, not the front-end
    syn = os.path.join(CSRC, "synth.hip")
    if force or _stale(SYNTH_LIB, [syn]):
        run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-shared", syn,
             "-o", SYNTH_LIB])
    return LIB


EXAMPLES = os.path.join(HERE, "..", "examples")


def build_examples() -> list:
    """The INTEGRATION.md host bindings as compiled programs (examples/*.cpp -> examples/_bin/),
    plain g++ against include/ and the in-tree library -- the way a reference node links it."""
    out_dir = os.path.join(EXAMPLES, "_bin")
    os.makedirs(out_dir, exist_ok=True)
    built = []
    for src in sorted(f for f in os.listdir(EXAMPLES) if f.endswith(".cpp")):
        s = os.path.join(EXAMPLES, src)
        exe = os.path.join(out_dir, src[:-4])
        if _stale(exe, [s, LIB, os.path.join(HERE, "..", "include", "ssf_frontend.h")]):
            subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-I", os.path.join(HERE, "..", "include"),
                            "-I", "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", s, "-L", OUT_DIR,
                            "-lssf_frontend", "-L", "/opt/rocm/lib", "-lamdhip64",
                            "-Wl,-rpath,$ORIGIN/../../ssf-slam_amd/ssf/_lib", "-Wl,-rpath,/opt/rocm/lib",
                            "-o", exe], check=True)
        built.append(exe)
    return built


def build_diag() -> str:
    """Diagnostic library (phase stamps in k_mask_pose, -DSSF_MASK_STAMPS) for
    tools/diag_mask_phases.py; never loaded by the product path unless SSF_LIB points at it."""
    out = os.path.join(OUT_DIR, "libssf_frontend_diag.so")
    objs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ_DIR, src.replace(".hip", "_diag.o"))
        extra = {"mask_pose.hip": ["-DSSF_MASK_STAMPS"], "mask_pose_f64.hip": ["-DSSF_MASK_STAMPS"],
                 "registration.hip": ["-DSSF_TABLE_STAMPS", "-DSSF_ASSOC_STAMPS"]}.get(src, [])
        subprocess.run([HIPCC, *FLAGS, *FILE_FLAGS.get(src, []), *extra, "-c", s, "-o", o], check=True)
        objs.append(o)
    subprocess.run([HIPCC, *FLAGS, "-shared", *objs, "-o", out], check=True)
    return out


def build_variant(name: str, defines: dict) -> str:
    """Experiment library (tools/ only, loaded through SSF_LIB): every source compiled with extra
    -D defines into ssf/_lib/libssf_frontend_<name>.so.  Never loaded by the product path."""
    out = os.path.join(OUT_DIR, f"libssf_frontend_{name}.so")
    extra = [f"-D{k}={v}" for k, v in defines.items()]
    objs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ_DIR, src.replace(".hip", f"_{name}.o"))
        subprocess.run([HIPCC, *FLAGS, *FILE_FLAGS.get(src, []), *extra, "-c", s, "-o", o], check=True)
        objs.append(o)
    subprocess.run([HIPCC, *FLAGS, "-shared", *objs, "-o", out], check=True)
    return out


if __name__ == "__main__":
    if "--diag" in sys.argv:
        print(build_diag())
    else:
        print(build(force="--force" in sys.argv, verbose=True))
