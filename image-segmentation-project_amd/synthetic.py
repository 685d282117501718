"""Seeded synthetic microscopy batches.

The reference trains on a private cell dataset (``dataset.py:17-66``: grayscale,
min-max normalised to [0, 1], binary ``mask > 0`` as float32 ``[1,H,W]``).  It is
not in the repo, so every benchmark and parity test here uses Gaussian "cells"
of the same shape and value range:

* 5-40 blobs per image, sigma 3-12 px (scaled with H/512 at other sizes),
* N(0, 0.1) noise, then min-max normalisation to [0, 1] (``dataset.py:41``),
* mask = blob support (exp(-r^2/2s^2) > 0.3 for any blob), ~20 % foreground.
"""
from __future__ import annotations

import numpy as np


def synthetic_cells(n: int, h: int, w: int, seed: int = 1234):
    """Return ``(images, masks)`` as float32 numpy arrays of shape [n,1,h,w]."""
    rng = np.random.default_rng(seed)
    images = np.empty((n, 1, h, w), np.float32)
    masks = np.empty((n, 1, h, w), np.float32)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    scale = max(h, w) / 512.0
    for i in range(n):
        img = np.zeros((h, w), np.float32)
        msk = np.zeros((h, w), bool)
        for _ in range(int(rng.integers(5, 41))):
            cy, cx = rng.uniform(0, h), rng.uniform(0, w)
            s = max(rng.uniform(3.0, 12.0) * max(scale, 0.25), 1.0)
            g = np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))
            img += rng.uniform(0.5, 1.0) * g
            msk |= g > 0.3
        img += rng.normal(0.0, 0.1, (h, w)).astype(np.float32)
        lo, hi = img.min(), img.max()
        images[i, 0] = (img - lo) / (hi - lo + 1e-8)
        masks[i, 0] = msk
    return images, masks


def random_batch(n: int, h: int, w: int, seed: int = 0):
    """i.i.d. N(0,1) images + Bernoulli(0.2) masks (throughput runs)."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, 1, h, w), dtype=np.float32)
    m = (rng.random((n, 1, h, w)) < 0.2).astype(np.float32)
    return x, m
