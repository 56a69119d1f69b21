"""HARRIS_SCORE in the CPU restatement (oracle), checked against an
independent numpy restatement of HarrisResponses (src/ORBextractor.cc:79-120).

The oracle's per-level keypoints (level coordinates, before the final
scaling) carry the Harris response it used for retainBest; numpy recomputes
it from the oracle's padded raw level with float32 scalar arithmetic (one
rounding per operation, the source's evaluation order).  Parity unpinned
against the reference binary: both are restatements.
"""
import numpy as np
import pytest

from orb_slam_amd import synth
from oracle_lib import RefExtractor

F = np.float32


def harris_np(padded, xs, ys):
    """HarrisResponses(img, pts, blockSize=7, HARRIS_K=0.04f) for keypoints
    at level coordinates (xs, ys); the level ROI sits at (16, 16)."""
    I = padded.astype(np.int64)
    X = xs.astype(np.int64) + 16
    Y = ys.astype(np.int64) + 16
    a = np.zeros(len(xs), np.int64)
    b = np.zeros_like(a)
    c = np.zeros_like(a)
    for i in range(-3, 4):
        for j in range(-3, 4):
            y, x = Y + i, X + j
            Ix = (I[y, x + 1] - I[y, x - 1]) * 2 + (I[y - 1, x + 1] - I[y - 1, x - 1]) + (I[y + 1, x + 1] - I[y + 1, x - 1])
            Iy = (I[y + 1, x] - I[y - 1, x]) * 2 + (I[y + 1, x - 1] - I[y - 1, x - 1]) + (I[y + 1, x + 1] - I[y - 1, x + 1])
            a += Ix * Ix
            b += Iy * Iy
            c += Ix * Iy
    scale = F(1.0) / (F(28) * F(255.0))
    s4 = scale * scale * scale * scale
    fa, fb, fc = a.astype(F), b.astype(F), c.astype(F)
    s = fa + fb
    return ((fa * fb - fc * fc) - (F(0.04) * s) * s) * s4


@pytest.mark.parametrize("kind,w,h,n,seed", [("texture", 640, 480, 1000, 1), ("noise", 333, 251, 500, 4),
                                             ("texture", 96, 80, 100, 3)])
def test_harris_responses_match_numpy(kind, w, h, n, seed):
    img = synth.texture_frame(w, h, seed) if kind == "texture" else synth.noise_frame(w, h, seed)
    ref = RefExtractor(n, score_type=0)
    kps, _ = ref(img)
    assert len(kps) > 0
    total = 0
    for lvl in range(8):
        lk = ref.level_keys(lvl)
        if len(lk) == 0:
            continue
        want = harris_np(ref.level(lvl), lk["x"], lk["y"])
        got = lk["response"]
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), \
            (lvl, np.count_nonzero(got != want))
        total += len(lk)
    assert total == len(kps)
    # the output keypoints carry the same responses, level-major
    want = np.concatenate([ref.level_keys(l)["response"] for l in range(8)])
    assert np.array_equal(kps["response"], want)


def test_harris_changes_selection_not_fast_candidates():
    """Harris only re-scores the FAST corners: every Harris-mode keypoint of
    a level is a FAST corner position of that level's cells, and the set of
    positions differs from FAST_SCORE's retained set on a textured frame."""
    img = synth.texture_frame(640, 480, 1)
    fk, _ = RefExtractor(1000, score_type=1)(img)
    hk, _ = RefExtractor(1000, score_type=0)(img)
    assert len(hk) == len(fk) == 1000
    assert not np.array_equal(hk[["x", "y"]], fk[["x", "y"]])
    assert np.all(np.mod(fk["response"], 1) == 0)
    assert np.any(np.mod(hk["response"], 1) != 0)
