"""Loop-closure registration timing: GPU voxel grid + ICP vs the CPU
oracle on the mapOptmization shapes -- the current keyframe (one plane cloud) against the local
map of 21 keyframes around the loop candidate, both through the 0.1 m voxel grid
(src/mapOptmization.cpp:200-236).  Synthetic scans (ssf/synth.py).  Prints one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ssf-slam_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from ssf import Frontend, loop, synth
    from oracle import oracle as O
    dev = torch.device("cuda", 0)
    fe = Frontend(64, device=0)
    sc = synth.Scene(0)
    R0, p0 = synth.ego_pose(0, 0)
    T0 = np.eye(4); T0[:3, :3] = R0.numpy(); T0[:3, 3] = p0.numpy()
    clouds = []
    for k in range(21):
        f = synth.scan(0, k, n_az=1875, scene=sc)
        pl = O.extract_planes(f["pos1"].numpy(), 64)
        R, p = synth.ego_pose(0, k)
        Tk = np.eye(4); Tk[:3, :3] = R.numpy(); Tk[:3, 3] = p.numpy()
        T = np.linalg.inv(T0) @ Tk
        x = pl.copy()
        x[:, :3] = (pl[:, :3].astype(np.float64) @ T[:3, :3].T + T[:3, 3]).astype(np.float32)
        clouds.append(x)
    cur = clouds[10].copy()
    cur[:, 0] += 0.5                                   # the drifted revisit
    local = np.concatenate(clouds)
    g_local = torch.from_numpy(local).to(dev)
    g_cur = torch.from_numpy(cur).to(dev)
    # warm-up
    tl = loop.voxel_grid_one(fe, g_local, 0.1)
    tc = loop.voxel_grid_one(fe, g_cur, 0.1)
    loop.icp(fe, tc, tl)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        tl = loop.voxel_grid_one(fe, g_local, 0.1)
        tc = loop.voxel_grid_one(fe, g_cur, 0.1)
        r = loop.icp(fe, tc, tl)
    torch.cuda.synchronize()
    gpu_ms = (time.perf_counter() - t0) / reps * 1e3
    t0 = time.perf_counter()
    vl = O.voxel_grid(local, 0.1)
    vc = O.voxel_grid(cur, 0.1)
    ro = O.icp(vc, vl)
    cpu_ms = (time.perf_counter() - t0) * 1e3
    print(json.dumps(dict(bench="loop_closure_registration", n_local=int(local.shape[0]),
                          n_local_voxel=int(tl.shape[0]), n_cur_voxel=int(tc.shape[0]),
                          gpu_ms=gpu_ms, cpu_oracle_ms=cpu_ms, cpu_threads=1,
                          iterations=r["iterations"], state=r["state"], fitness=r["fitness"],
                          oracle_iterations=ro["iterations"],
                          dx=float(r["T"][0, 3]), oracle_dx=float(ro["T"][0, 3]))))


if __name__ == "__main__":
    main()
