"""Bitwise comparison of two .npz dumps (same keys): prints, per key, whether every element is
identical (floats compared as raw bits) and the count of differing elements."""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
for k in a.files:
    x, y = a[k], b[k]
    if x.dtype.kind == "f":
        x, y = x.view(np.uint32 if x.itemsize == 4 else np.uint64), y.view(np.uint32 if y.itemsize == 4 else np.uint64)
    same = x.shape == y.shape and np.array_equal(x, y)
    nd = int((x != y).sum()) if x.shape == y.shape else -1
    print(f"{k}: identical={same} differing={nd} size={x.size}")
    if not same and x.shape == y.shape and x.ndim == 2:
        cols = sorted(set(np.nonzero(x != y)[1].tolist()))
        print(f"  differing columns {cols}")
        if a[k].dtype.kind == "f":
            for c in cols[:8]:
                d = np.abs(a[k][:, c] - b[k][:, c])
                rel = d / np.maximum(np.abs(a[k][:, c]), 1e-300)
                print(f"  col {c}: max abs diff {d.max():.3e}, max rel {rel.max():.3e}")
