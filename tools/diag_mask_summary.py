"""Summary of a tools/diag_mask_frames.py dump: mean frame cycles, per-pass cycles and the pass
tails (diagnostic build slots, see mask_pose.hip SSF_MASK_STAMPS)."""
import sys

import numpy as np

for p in sys.argv[1:]:
    o = np.load(p)["out"]
    km, em = o[:, 19].sum(), o[:, 20].sum()
    st = o[:, 26:32]
    d = np.diff(np.concatenate([np.zeros((len(o), 1)), st], 1), axis=1)
    print(f"{p}: frame mean {st[:, 5].mean():.4e} max {st[:, 5].max():.4e}; lloyd/pass {d[:, 2].sum() / km:.0f}; "
          f"em/pass {d[:, 4].sum() / em:.0f}")
    names = ["pass0", "kmeans++", "lloyd", "gmm_init", "em", "final+mask"]
    print("   phases (mean cycles): " + ", ".join(f"{k} {v:.3e}" for k, v in zip(names, d.mean(0))))
