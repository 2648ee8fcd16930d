"""HBM traffic per launch of one kernel from two rocprofv3 counter passes (bench.py roofline.traffic).

Collect the passes separately (FETCH_SIZE needs 3 TCC counters, WRITE_SIZE 2; one run cannot
hold both), on the bench command whose roofline they annotate:

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline
    python tools/pmc_traffic.py gpurun_out/pmc_fetch/f_counter_collection.csv \
        gpurun_out/pmc_write/w_counter_collection.csv --bench-log gpurun_out/pmc_fetch.log \
        --out profiles/r01_k_mask_pose_traffic.json

Units and corrections (/opt/skills/guides/MI355X_MICROARCH.md, "HBM [CDNA4]"): FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE tallies wide coalesced streaming reads at half their
bytes, so it is doubled; WRITE_SIZE is taken as is.  The first launch (cold caches, first touch)
is reported but excluded from the per-launch mean.
"""
from __future__ import annotations

import argparse
import csv
import json


def launches(path, kernel):
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [float(r["Counter_Value"]) for r in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--kernel", default="k_mask_pose")
    ap.add_argument("--bench-log", help="stdout of the profiled bench run (its JSON line names the config)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch = launches(a.fetch_csv, a.kernel)
    write = launches(a.write_csv, a.kernel)
    if len(fetch) < 2 or len(write) < 2:
        raise SystemExit(f"need >= 2 launches of {a.kernel} in each pass ({len(fetch)}, {len(write)})")
    f_mean = sum(fetch[1:]) / (len(fetch) - 1)
    w_mean = sum(write[1:]) / (len(write) - 1)
    out = {
        "kernel": a.kernel,
        "fetch_size_kib": fetch,
        "write_size_kib": write,
        "read_bytes_per_launch": 2.0 * f_mean * 1024.0,
        "write_bytes_per_launch": w_mean * 1024.0,
        "traffic_bytes_per_launch": 2.0 * f_mean * 1024.0 + w_mean * 1024.0,
        "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half tally of wide streaming reads) + WRITE_SIZE KiB x 1024; "
                      "first launch excluded",
    }
    if a.bench_log:
        for line in open(a.bench_log):
            if line.startswith("{"):
                d = json.loads(line)
                out["config"] = {k: d["config"][k] for k in ("sequences_per_gpu", "points_per_frame")}
                k = d["kernels"].get(a.kernel)
                if k:
                    out["algorithmic_bytes_per_launch"] = k["bytes"]
                    out["passes_per_frame"] = k.get("passes_per_frame")
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if not isinstance(v, list)}, indent=1))


if __name__ == "__main__":
    main()
