"""f64 VALU work per k_mask_pose launch from one rocprofv3 counter pass (bench.py roofline_f64).

    rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 \
        SQ_INSTS_VALU_TRANS_F64 --output-format csv -d gpurun_out/pmc_f64 -o d -- python bench.py --serial ...
    python tools/pmc_f64.py gpurun_out/pmc_f64/d_counter_collection.csv --bench-log LOG \
        --out profiles/r02_k_mask_pose_f64.json

The SQ_INSTS_VALU_*_F64 counters count wave-level instructions; one f64 instruction of a 64-lane
wave is 64 lane operations, an FMA counting 2 FLOPs.  Lanes masked off by exec are counted as
issued, so this is an ISSUE figure (what the VALU spent), not useful lanes.  Peak: 78.6 TFLOP/s
FP64 vector (MI355X spec)."""
from __future__ import annotations

import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel", default="k_mask_pose")
    ap.add_argument("--bench-log")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    per = defaultdict(dict)                                   # dispatch -> counter -> value
    for r in csv.DictReader(open(a.csv)):
        if a.kernel in r["Kernel_Name"]:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(per)
    if len(ids) < 2:
        raise SystemExit(f"need >= 2 launches of {a.kernel}, got {len(ids)}")
    w = {"SQ_INSTS_VALU_FMA_F64": 2.0, "SQ_INSTS_VALU_MUL_F64": 1.0, "SQ_INSTS_VALU_ADD_F64": 1.0,
         "SQ_INSTS_VALU_TRANS_F64": 1.0}
    flops = [64.0 * sum(w[c] * per[i].get(c, 0.0) for c in w) for i in ids]
    out = {"kernel": a.kernel, "counters_per_launch": [per[i] for i in ids],
           "f64_flops_per_launch": sum(flops[1:]) / (len(flops) - 1),
           "rule": "64 lanes x (2 FMA + MUL + ADD + TRANS) wave instructions; first launch excluded"}
    if a.bench_log:
        for line in open(a.bench_log):
            if line.startswith("{"):
                d = json.loads(line)
                out["config"] = {k: d["config"][k] for k in ("sequences_per_gpu", "points_per_frame",
                                                              "mask_before_features")}
                out["lib_sha16"] = d.get("lib_sha16")        # the build these counters measured
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "counters_per_launch"}, indent=1))


if __name__ == "__main__":
    main()
