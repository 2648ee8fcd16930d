"""Print a compact summary of bench JSON lines / bench_features outputs (last JSON line of each file)."""
import glob
import json
import sys

for pat in sys.argv[1:]:
    for f in sorted(glob.glob(pat)):
        try:
            d = json.loads([l for l in open(f) if l.startswith("{")][-1])
        except (IndexError, ValueError, OSError) as e:
            print(f, "-", e)
            continue
        if "kernel_ms" in d:
            print(f, d.get("tag"), {k: round(v, 4) for k, v in d["kernel_ms"].items()},
                  "sum", round(sum(d["kernel_ms"].values()), 4))
        else:
            print(f, round(d.get("value", 0), 1), d.get("unit"), "ms/step", round(d.get("ms_per_step", 0), 3),
                  "gather", d.get("gather_check"))
