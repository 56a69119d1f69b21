"""Deterministic synthetic mono8 inputs.

The reference ships no images (its example rosbag is an external download,
README.md:150), so tests and the benchmark use generated frames:

* texture_frame -- smoothed uniform noise, contrast-stretched, plus random
  axis-aligned rectangles: FAST density of a few percent with saturated and
  starved cells.
* noise_frame   -- pure uniform noise (FAST fires almost everywhere).
* flat_frame    -- constant 128 (FAST finds nothing: threshold-7 fallback and
  the empty-level paths).
* sequence      -- "TUM-style" camera motion: frame k is a w x h window of a
  larger texture; 300 distinct window offsets per period (sequence_offset).
"""
import numpy as np


def _rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def _box5(a):
    """5x5 box mean with edge replication (float64)."""
    p = np.pad(a.astype(np.float64), 2, mode="edge")
    c = np.cumsum(np.cumsum(p, axis=0), axis=1)
    c = np.pad(c, ((1, 0), (1, 0)))
    h, w = a.shape
    s = c[5:5 + h, 5:5 + w] - c[0:h, 5:5 + w] - c[5:5 + h, 0:w] + c[0:h, 0:w]
    return s / 25.0


def texture_frame(w, h, seed, n_rects=200):
    r = _rng(seed)
    base = _box5(r.integers(0, 256, size=(h, w)))
    lo, hi = base.min(), base.max()
    img = ((base - lo) * (255.0 / max(hi - lo, 1e-9))).astype(np.uint8)
    for _ in range(n_rects):
        x0 = int(r.integers(0, w))
        y0 = int(r.integers(0, h))
        rw = int(r.integers(4, max(5, w // 8)))
        rh = int(r.integers(4, max(5, h // 8)))
        img[y0:y0 + rh, x0:x0 + rw] = np.uint8(r.integers(0, 256))
    return img


def noise_frame(w, h, seed):
    return _rng(seed).integers(0, 256, size=(h, w), dtype=np.uint8)


def flat_frame(w, h, value=128):
    return np.full((h, w), value, dtype=np.uint8)


SEQ_PERIOD = 300     # a 300-frame sequence at 30 Hz


def sequence_offset(k):
    """Window offset (dx, dy) of frame k: a horizontal pan of +-2 px per frame
    (a triangle wave over 0..40) while the camera drifts down one pixel every
    five frames.  The 300 offsets of a period are pairwise distinct (within a
    run of five frames dy is constant and the triangle values differ), so
    a 300-frame sequence has no repeated frame; longer runs cycle."""
    k %= SEQ_PERIOD
    t = k % 40
    return (2 * t if t < 20 else 2 * (40 - t)), k // 5


def sequence(w, h, n_frames, seed):
    """n_frames x h x w uint8 frames of one synthetic camera sequence."""
    big = texture_frame(w + 40, h + SEQ_PERIOD // 5, seed, n_rects=260)
    out = np.empty((n_frames, h, w), dtype=np.uint8)
    for k in range(n_frames):
        dx, dy = sequence_offset(k)
        out[k] = big[dy:dy + h, dx:dx + w]
    return out
