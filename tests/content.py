"""Synthetic RGB888 content beyond band4, for parity stress (SURVEY.md §8(d):
"add a noise stress ... and a static best case").  Each generator is a pure
function of (w, h, t, seed); all of them are plain numpy, the oracle and the
GPU path see the same bytes.

kinds:
  noise    uniform random RGB every frame: no copy blocks, full searches
  static   band4 frame 0 repeated: copy blocks and output_cache carry-over
  black    RGB (0, 0, 0): Y = 16, flat, every SAD ties
  white    RGB (255, 255, 255): Y = 271, the 9-bit luma maximum
  ties     a flat grey field with +-3 noise on 5 % of the pixels: near-equal
           SADs everywhere, so the order-dependent tie rules decide
  pan      band4 frame 0 shifted 40 px right and 24 px down per frame (beyond
           the +-31 px search reach) with a scene cut to noise at t = 3
  gradient smooth ramps moving by a fractional amount: sub-pel candidates win
"""
from __future__ import annotations

import numpy as np

KINDS = ("noise", "static", "black", "white", "ties", "pan", "gradient")


def _band4(w, h, t, seed=1234):
    from oracle import oracle as orc

    return orc.make_frame(w, h, t, seed)


def make(kind: str, w: int, h: int, t: int, seed: int = 7) -> np.ndarray:
    rng = np.random.default_rng(seed * 1000003 + t)
    if kind == "noise":
        return rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    if kind == "static":
        return _band4(w, h, 0)
    if kind == "black":
        return np.zeros((h, w, 3), np.uint8)
    if kind == "white":
        return np.full((h, w, 3), 255, np.uint8)
    if kind == "ties":
        img = np.full((h, w, 3), 128, np.int16)
        mask = rng.random((h, w)) < 0.05
        img[mask] += rng.integers(-3, 4, (int(mask.sum()), 1), dtype=np.int16)
        return img.clip(0, 255).astype(np.uint8)
    if kind == "pan":
        if t >= 3:
            return rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        base = _band4(w, h, 0)
        return np.roll(base, (24 * t, 40 * t), axis=(0, 1)).copy()
    if kind == "gradient":
        y, x = np.mgrid[0:h, 0:w].astype(np.float64)
        s = 0.5 * t  # half a pixel per frame
        r = (x + s) * 255.0 / max(w, 1)
        g = (y + s) * 255.0 / max(h, 1)
        b = ((x + y + 2 * s) * 127.0 / max(w + h, 1)) + 64
        return np.stack([r, g, b], -1).astype(np.uint8)
    raise ValueError(kind)
