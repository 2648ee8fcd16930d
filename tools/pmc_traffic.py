"""HBM traffic per launch of every kernel from two rocprofv3 counter passes (bench.py `traffic`).

Collect the passes separately (FETCH_SIZE needs 3 TCC counters, WRITE_SIZE 2; one run cannot
hold both), on a serial bench command (one stream, so every launch is that kernel alone):

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python bench.py --serial ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python bench.py --serial ...
    python tools/pmc_traffic.py gpurun_out/pmc_fetch/f_counter_collection.csv \
        gpurun_out/pmc_write/w_counter_collection.csv --bench-log gpurun_out/pmc_fetch.log \
        --out profiles/r02_traffic.json

Units and corrections (/opt/skills/guides/MI355X_MICROARCH.md, "HBM [CDNA4]"): FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE tallies wide coalesced streaming reads at half their
bytes, so it is doubled; WRITE_SIZE is taken as is.  The first launch of each kernel (cold
caches, first touch) is reported but excluded from the per-launch mean.
"""
from __future__ import annotations

import argparse
import csv
import json
from collections import defaultdict

KERNELS = ("k_mask_pose_f64", "k_mask_pose", "k_feat_wave_reg", "k_feat_wave_run", "k_feat_chunk_reg", "k_feat_chunk_flagged", "k_feat_chunk", "k_feat_select", "k_bin_count", "k_bin_scan", "k_bin_curv", "k_select",
           "k_plane_table_sorted", "k_associate_strips", "k_associate_lds", "k_associate_sorted", "k_solve")


def launches(path):
    """{kernel: [counter value per dispatch, in dispatch order]} for the front-end kernels"""
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    out = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        if "<true," in name and ("k_feat_chunk" in name or "k_feat_wave" in name or "k_bin_curv" in name):
            continue                    # the debug instantiation (bench's kernel-pass byte counts)
        if "k_feat_debug" in name:
            continue
        for k in KERNELS:
            if k + "(" in name or k + "<" in name or name.startswith(k) or (" " + k) in name:
                out[k].append(float(r["Counter_Value"]))
                break
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--bench-log", help="stdout of the profiled bench run (its JSON line names the config)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch, write = launches(a.fetch_csv), launches(a.write_csv)
    out = {"correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half tally of wide streaming reads) + "
                         "WRITE_SIZE KiB x 1024; first launch of each kernel excluded",
           "kernels": {}}
    for k in KERNELS:
            f, w = fetch.get(k, []), write.get(k, [])
            if len(f) < 2 or len(w) < 2:
                continue
            fm = sum(f[1:]) / (len(f) - 1)
            wm = sum(w[1:]) / (len(w) - 1)
            out["kernels"][k] = dict(launches=len(f), read_bytes_per_launch=2.0 * fm * 1024.0,
                                     write_bytes_per_launch=wm * 1024.0,
                                     traffic_bytes_per_launch=2.0 * fm * 1024.0 + wm * 1024.0)
    if a.bench_log:
        for line in open(a.bench_log):
            if line.startswith("{"):
                d = json.loads(line)
                out["config"] = {k: d["config"][k] for k in ("sequences_per_gpu", "points_per_frame",
                                                              "mask_before_features")}
                out["config"]["layout"] = d["config"].get("layout", "azimuth")
                out["lib_sha16"] = d.get("lib_sha16")        # the build these counters measured
                for k, v in d.get("kernels", {}).items():
                    if k in out["kernels"] and "bytes" in v:
                        out["kernels"][k]["algorithmic_bytes_per_launch"] = v["bytes"]
                        out["kernels"][k]["traffic_over_algorithmic"] = (
                            out["kernels"][k]["traffic_bytes_per_launch"] / v["bytes"])
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
