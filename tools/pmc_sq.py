"""Per-kernel SQ / TA counter table from rocprofv3 --pmc passes (issue / stall / LDS counters).

Each pass is its own run of the same serial bench command (rocprofv3 does not split counters
over passes; at most 8 SQ and 2 TA counters per run, MI355X_MICROARCH.md):

    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... --output-format csv -d gpurun_out/sq1 -o p -- python bench.py --serial ...
    python tools/pmc_sq.py gpurun_out/sq1/p_counter_collection.csv gpurun_out/sq2/... --out profiles/r04_sq.json

Units (rocprofv3 -L descriptions): SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_* count quad-cycles
per wave (x4 -> cycles); SQ_BUSY_CYCLES is clock cycles per shader engine; SQ_INSTS_* count
wave-instructions.  Counters are summed over every hardware instance of a dispatch (the CSV has
one row per dispatch and counter after rocprofv3's own reduction).  The first launch of each
kernel is excluded from the mean (cold caches, code load).  Derived per launch:
  instructions per wave (VALU / SALU / LDS / VMEM), VALU issue share of the wave-cycles,
  stall shares (WAIT_INST_ANY: instruction-issue stalls; WAIT_ANY: waits on counters / barriers).
"""
from __future__ import annotations

import argparse
import csv
import json
from collections import defaultdict

KERNELS = ("k_mask_pose_f64", "k_mask_pose", "k_bin_count", "k_bin_scan", "k_bin_curv", "k_select",
           "k_feat_wave_reg", "k_feat_wave_run", "k_feat_chunk_reg", "k_feat_chunk_flagged", "k_feat_chunk", "k_feat_select", "k_plane_table_sorted", "k_associate_strips",
           "k_associate_strips_soa", "k_solve", "k_kabsch_f32")


def kernel_of(name):
    base = name.split("(")[0].split("<")[0].strip()
    base = base.split("::")[-1] if "::" in base else base
    for k in KERNELS:
        if base == k or base.endswith(" " + k):
            return k
    return None


def read(paths):
    """{kernel: {counter: [value per dispatch in dispatch order]}}"""
    out = defaultdict(lambda: defaultdict(list))
    for p in paths:
        rows = list(csv.DictReader(open(p)))
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        mine = defaultdict(lambda: defaultdict(list))
        for r in rows:
            k = kernel_of(r["Kernel_Name"])
            if k:
                mine[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in mine.items():          # a counter repeated in a later pass: the first pass's
            for c, v in cs.items():
                if c not in out[k]:
                    out[k][c] = v
    return out


def mean_wo_first(v):
    return sum(v[1:]) / (len(v) - 1) if len(v) > 1 else (v[0] if v else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--out", required=True)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    data = read(a.csv)
    res = {"source": [p for p in a.csv], "note": a.note,
           "units": "SQ_INSTS_*: wave-instructions per launch; SQ_WAVE_CYCLES / SQ_WAIT_* / "
                    "SQ_ACTIVE_INST_*: quad-cycles summed over waves (x4 = cycles); first launch excluded",
           "kernels": {}}
    for k, cs in sorted(data.items()):
        m = {c: mean_wo_first(v) for c, v in cs.items()}
        d = {"launches": max(len(v) for v in cs.values()), "per_launch": m}
        waves = m.get("SQ_WAVES")
        if waves:
            per = {}
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                      "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH", "SQ_INSTS_SMEM",
                      "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                      "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_INT32", "SQ_INSTS_LDS_LOAD"):
                if m.get(c) is not None:
                    per[c.replace("SQ_INSTS_", "")] = m[c] / waves
            for c in ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_ADDR_CONFLICT", "SQ_LDS_IDX_ACTIVE",
                      "SQ_LDS_UNALIGNED_STALL"):       # LDS cycle counters, per wave
                if m.get(c) is not None:
                    per[c.replace("SQ_", "")] = m[c] / waves
            if m.get("SQ_WAVE_CYCLES") is not None:
                per["WAVE_CYCLES"] = 4.0 * m["SQ_WAVE_CYCLES"] / waves
            d["per_wave"] = per
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            sh = {}
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_ANY",
                      "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_LDS"):
                if m.get(c) is not None:
                    sh[c.replace("SQ_", "")] = m[c] / wc
            d["share_of_wave_cycles"] = sh
        res["kernels"][k] = d
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    for k, d in res["kernels"].items():
        print(k, json.dumps({kk: round(v, 3) for kk, v in d.get("per_wave", {}).items()}),
              json.dumps({kk: round(v, 3) for kk, v in d.get("share_of_wave_cycles", {}).items()}))


if __name__ == "__main__":
    main()
