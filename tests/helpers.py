"""Shared synthetic inputs for the tests (seeded, deterministic)."""
import functools

import numpy as np


@functools.lru_cache(maxsize=None)
def frame(seq, k, n_rows=64, n_az=600):
    from ssf import synth
    f = synth.scan(seq, k, n_rows=n_rows, n_az=n_az, scene=_scene(seq))
    return f["pos1"].numpy(), f["flow"].numpy(), f["s_fg_mask"].numpy()


@functools.lru_cache(maxsize=None)
def _scene(seq):
    from ssf import synth
    return synth.Scene(seq)


def shuffled(pts, seed):
    """Same cloud in a different arrival order (exercises the stable per-ring partition)."""
    rng = np.random.default_rng(seed)
    return pts[rng.permutation(pts.shape[0])]
