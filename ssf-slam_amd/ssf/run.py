"""python -m ssf.run DATASET_PATH [--tum traj.txt]: replay an npz scene-flow sequence through the
device front-end as launch/*.launch wires the reference's nodes (PointCloudOdometry_noSeg ->
frameFeature -> lidarOdometry_onlyPC [-> mapOptmization loop closure]) and write /frame_odom2 as a
TUM trajectory."""
from __future__ import annotations

import argparse
import json

import torch


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m ssf.run")
    ap.add_argument("dataset_path", help="directory of npz frames with pos1 and gt (flow)")
    ap.add_argument("--tum", default=None, help="TUM output (stamp x y z qx qy qz qw)")
    ap.add_argument("--rows", type=int, default=64, choices=[16, 64])
    ap.add_argument("--solver", default="ceres_lm", choices=["ceres_lm", "gn"])
    ap.add_argument("--iters", type=int, default=None)
    ap.add_argument("--seed", type=int, default=None, help="np.random.seed for the GMM k-means++")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--map-tum", default=None,
                    help="also run mapOptmization (loop closure) and write its RESULT_PATH TUM file")
    a = ap.parse_args(argv)
    from .nodes import run_sequence
    torch.cuda.set_device(a.device)
    res = run_sequence(a.dataset_path, a.tum, n_rows=a.rows, solver=a.solver, max_iter=a.iters,
                       seed=a.seed, map_tum_path=a.map_tum)
    print(json.dumps({"frames": int(res["odom1"].shape[0]), "odom2_poses": int(res["odom2"].shape[0]),
                      "final_t": res["odom2"][-1, 0:3].tolist() if len(res["odom2"]) else None,
                      "loops": len(res["loops"])}))


if __name__ == "__main__":
    main()
