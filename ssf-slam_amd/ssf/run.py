"""python -m ssf.run DATASET_PATH [--launch noSeg] [--tum traj.txt]: replay an npz scene-flow
sequence through the device front-end as one of the reference's launch files wires its nodes
(launch/run_onlyPC.launch, run_noSeg.launch, run_Seg.launch; ssf.nodes.LAUNCH_GRAPHS) and append
/frame_odom2 to a TUM trajectory (optionally with mapOptmization's loop closure)."""
from __future__ import annotations

import argparse
import json

import torch


def main(argv=None):
    from .nodes import LAUNCH_GRAPHS
    ap = argparse.ArgumentParser(prog="python -m ssf.run")
    ap.add_argument("dataset_path", help="directory of npz frames (pos1, gt = flow, s_fg_mask)")
    ap.add_argument("--launch", default="noSeg", choices=sorted(LAUNCH_GRAPHS),
                    help="node graph of launch/run_<launch>.launch")
    ap.add_argument("--tum", default=None, help="TUM output (stamp x y z qx qy qz qw), appended")
    ap.add_argument("--truncate", action="store_true", help="empty the TUM files first")
    ap.add_argument("--rows", type=int, default=64, choices=[16, 64])
    ap.add_argument("--solver", default="ceres_lm", choices=["ceres_lm", "gn"])
    ap.add_argument("--iters", type=int, default=None)
    ap.add_argument("--seed", type=int, default=None, help="np.random.seed for the GMM k-means++")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--map-tum", default=None,
                    help="also run mapOptmization (loop closure) and write its RESULT_PATH TUM file")
    a = ap.parse_args(argv)
    from .nodes import run_sequence
    import os
    import sys
    if a.tum and os.path.exists(a.tum) and not a.truncate:
        print(f"ssf.run: appending to the existing {a.tum} (the reference's std::ios::app); "
              f"--truncate starts a new file", file=sys.stderr)
    torch.cuda.set_device(a.device)
    res = run_sequence(a.dataset_path, a.tum, n_rows=a.rows, solver=a.solver, max_iter=a.iters,
                       seed=a.seed, launch=a.launch, map_tum_path=a.map_tum,
                       truncate_results=a.truncate)
    print(json.dumps({"launch": a.launch, "tum": a.tum, "tum_mode": "truncate" if a.truncate else "append",
                      "frames": len(res["stamps"]),
                      "odom1_poses": int(res["odom1"].shape[0]),
                      "odom2_poses": int(res["odom2"].shape[0]),
                      "final_t": res["odom2"][-1, 0:3].tolist() if len(res["odom2"]) else None,
                      "loops": len(res["loops"])}))


if __name__ == "__main__":
    main()
