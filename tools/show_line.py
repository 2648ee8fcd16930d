"""Print the headline fields and the per-kernel table of bench.py JSON lines (one file each)."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, "value", round(d.get("value", 0), 1), d.get("unit"), "ms/step", round(d.get("ms_per_step", 0), 3),
          "roofline", (d.get("roofline") or {}).get("frac"), "ns", d.get("north_star_kernels_hbm_frac"))
    for n, v in (d.get("kernels") or {}).items():
        print("   %-24s" % n, {a: (round(b, 4) if isinstance(b, float) else b) for a, b in v.items()
                              if a in ("launches", "ms", "gbs", "frac", "traffic_frac")})
