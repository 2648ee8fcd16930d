"""Print the key numbers of bench.py JSON lines (files given on the command line)."""
import json
import sys

for path in sys.argv[1:]:
    L = [l for l in open(path) if l.startswith("{")]
    if not L:
        print(path, "no JSON line")
        continue
    d = json.loads(L[-1])
    print(path, "value", round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "gen_s", d.get("data_gen_s"),
          "passes", round(d.get("mask_passes_per_frame") or 0, 2), "gather", d.get("gather_check"))
    r = d.get("roofline") or {}
    print("  roofline", r.get("kernel"), round(r.get("frac", 0), 4), "f64", (d.get("roofline_f64") or {}).get("frac"))
    for k, v in (d.get("kernels") or {}).items():
        print("   %-22s n=%d ms=%.4f" % (k, v["launches"], v["ms"]),
              ("GB/s=%.0f frac=%.3f" % (v["gbs"], v["frac"])) if "gbs" in v else "")
    print("  overlapped", {k: round(v, 3) for k, v in (d.get("overlapped_event_ms") or {}).items()})
    if d.get("cpu_baseline"):
        c = d["cpu_baseline"]
        print("  cpu", round(c["value"], 2), c["cores"], {k: round(v["value"], 2) for k, v in c.get("legs", {}).items()})
