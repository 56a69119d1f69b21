"""An independent numpy restatement of OpenCV 2.4's FAST-9/16 with non-max
suppression (features2d/src/fast.cpp: FAST_t<16> and cornerScore<16>), the
detector ORBextractor runs per cell (src/ORBextractor.cc:607, :613), against
the oracle's restatement (oracle/ref_extract.cpp cv24_fast16).

The oracle follows OpenCV's loop structure (the tab[] pre-tests, the 25-entry
extended circle with a run counter, cornerScore's pruned min/max sweeps
starting from the threshold).  This restatement is written from the
definitions instead, vectorised over the image:

* d_k = v - p_k over the 16 Bresenham-circle pixels (radius 3);
* a pixel at row i in [3, rows - 4], column j in [3, cols - 4] is a corner
  at threshold t when 9 contiguous circle pixels are all darker than v - t
  or all brighter than v + t, i.e. max(A, B) > t with
  A = max_k min(d_k .. d_k+8), B = max_k min(-d_k .. -d_k+8) (indices mod 16);
* its score is max(t, A, B) - 1 (cornerScore returns the largest threshold
  at which the pixel is still a corner, minus one);
* non-max suppression keeps a corner whose score is strictly greater than
  the scores of its 8 neighbours (0 where not a corner);
* keypoints come out in raster order, cv::KeyPoint(j, i, 7, -1, score).
"""
import ctypes

import numpy as np
import pytest

from orb_slam_amd import synth
from oracle_lib import KEYPOINT, load

RING = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
        (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]   # (dx, dy)


def fast_np(img, t):
    img = np.asarray(img, np.int32)
    rows, cols = img.shape
    if rows < 7 or cols < 7:
        return np.zeros(0, KEYPOINT)
    t = min(max(int(t), 0), 255)
    v = img[3:rows - 3, 3:cols - 3]
    d = np.stack([v - img[3 + dy:rows - 3 + dy, 3 + dx:cols - 3 + dx] for dx, dy in RING])   # (16, h, w)
    dd = np.concatenate([d, d[:8]])
    arc_min = np.stack([dd[k:k + 9].min(axis=0) for k in range(16)])
    arc_max = np.stack([dd[k:k + 9].max(axis=0) for k in range(16)])
    A = arc_min.max(axis=0)
    B = (-arc_max).max(axis=0)
    corner = np.maximum(A, B) > t
    score = np.where(corner, np.maximum(np.maximum(A, B), t) - 1, 0)
    # neighbours of the scored region (rows / cols 3 .. n-4); pixels outside it
    # (the border ring of the cell) have no score
    S = np.zeros((rows, cols), np.int32)
    S[3:rows - 3, 3:cols - 3] = score
    c = S[3:rows - 3, 3:cols - 3]
    keep = corner.copy()
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dx == 0 and dy == 0:
                continue
            keep &= c > S[3 + dy:rows - 3 + dy, 3 + dx:cols - 3 + dx]
    ii, jj = np.nonzero(keep)
    out = np.zeros(len(ii), KEYPOINT)
    out["x"] = jj + 3
    out["y"] = ii + 3
    out["size"] = 7
    out["angle"] = -1
    out["response"] = c[ii, jj]
    out["octave"] = 0
    out["class_id"] = -1
    return out


def oracle_fast(img, t):
    L = load()
    img = np.ascontiguousarray(img, np.uint8)
    rows, cols = img.shape
    cap = rows * cols
    out = np.zeros(cap, KEYPOINT)
    n = ctypes.c_int(0)
    r = L.orbx_ref_fast_cell(img.ctypes.data_as(ctypes.c_void_p), cols, rows, cols, int(t),
                             out.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(n))
    assert r == 0
    return out[:n.value]


def images():
    r = np.random.default_rng(7)
    yield "noise", r.integers(0, 256, (48, 64), dtype=np.uint8)
    yield "texture", synth.texture_frame(128, 81, 11)[:, :]
    yield "frame-cell", synth.texture_frame(640, 480, 2000)[100:181, 200:328]
    flat = np.full((40, 40), 120, np.uint8)
    yield "flat", flat
    spots = flat.copy()
    spots[10, 10] = 250          # a bright point: 16 of 16 ring pixels darker
    spots[20, 25] = 0            # a dark point
    spots[30:33, 12:15] = 200    # a small square: its corners
    yield "spots", spots
    pair = flat.copy()
    pair[10, 10:12] = 250        # two equal neighbouring corners: strict NMS keeps neither
    pair[25, 20] = 250
    pair[26, 21] = 240           # a weaker neighbour on the diagonal: only the stronger stays
    yield "pair", pair
    levels = (r.integers(0, 4, (60, 72)) * 80).astype(np.uint8)   # coarse levels: many equal scores
    yield "levels", levels


@pytest.mark.parametrize("t", [1, 7, 20, 60])
def test_fast_matches_oracle(t):
    for name, img in images():
        got = fast_np(img, t)
        want = oracle_fast(img, t)
        assert len(got) == len(want), (name, t, len(got), len(want))
        for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
            assert np.array_equal(got[f], want[f]), (name, t, f)


def test_fast_known_corners():
    """The restatement itself on hand-built cases: an isolated bright pixel
    on a flat background scores (250 - 120) - 1 = 129 at any threshold below
    130 and is the only keypoint; the same pixel is no corner at 130."""
    img = np.full((21, 21), 120, np.uint8)
    img[10, 10] = 250
    k = fast_np(img, 20)
    assert len(k) == 1 and (k["x"][0], k["y"][0], k["response"][0]) == (10, 10, 129)
    assert len(fast_np(img, 130)) == 0
