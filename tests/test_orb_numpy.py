"""Independent numpy restatements of ORBextractor's orientation and
descriptor (A7 / A8 / A10), against the oracle on whole extractions.

Written from the reference's definitions, not from the oracle's code:

* umax (ORBextractor::ORBextractor, src/ORBextractor.cc:493-511):
  cvRound(sqrt(hp2 - v^2)) for v <= vmax, then the symmetric fill;
* IC_Angle (src/ORBextractor.cc:127-152): integer moments m_10, m_01 over
  the circular patch of the unblurred level, then cv::fastAtan2 (the float32
  restatement of tests/test_cv24_numpy.py);
* computeOrbDescriptor (src/ORBextractor.cc:157-195): angle * (float)(CV_PI
  / 180), a = cos, b = sin as correctly rounded float32 values (the glibc
  cosf / sinf of the reference's era of this image),
  sample offsets cvRound(x b + y a), cvRound(x a - y b) in float32 with each
  operation rounded (ISO evaluation, the default orbx_set_fp_contract(0)),
  round half to even, 256 comparisons t0 < t1 of the blurred level in
  bit_pattern_31_ order, 8 bits per byte, LSB first.

The pattern is the product's data copy (orb_slam_amd/csrc/orbx_pattern.inc).
"""
import re
from pathlib import Path

import numpy as np
import pytest

from orb_slam_amd import synth
from oracle_lib import RefExtractor
from test_cv24_numpy import fast_atan2_np

F32 = np.float32
HP = 15          # HALF_PATCH_SIZE (src/ORBextractor.cc:76)
EDGE = 16        # the padded level's border (oracle / product layout)
ROOT = Path(__file__).resolve().parents[1]


def pattern():
    text = (ROOT / "orb_slam_amd" / "csrc" / "orbx_pattern.inc").read_text()
    q = [tuple(int(v) for v in m) for m in re.findall(r"\{(-?\d+),(-?\d+),(-?\d+),(-?\d+)\}", text)]
    assert len(q) == 256
    return np.array(q, np.int64)   # (x1, y1, x2, y2) per pair


def umax_np():
    hp2 = HP * HP
    vmax = int(np.floor(HP * np.sqrt(2.0) / 2 + 1))
    vmin = int(np.ceil(HP * np.sqrt(2.0) / 2))
    u = np.zeros(HP + 1, np.int64)
    for v in range(vmax + 1):
        u[v] = int(np.rint(np.sqrt(float(hp2 - v * v))))
    v0 = 0
    for v in range(HP, vmin - 1, -1):
        while u[v0] == u[v0 + 1]:
            v0 += 1
        u[v] = v0
        v0 += 1
    return u


def ic_angle_np(raw, x, y, umax):
    cy, cx = int(np.rint(F32(y))) + EDGE, int(np.rint(F32(x))) + EDGE
    img = raw.astype(np.int64)
    m10 = int((np.arange(-HP, HP + 1) * img[cy, cx - HP:cx + HP + 1]).sum())
    m01 = 0
    for v in range(1, HP + 1):
        d = int(umax[v])
        u = np.arange(-d, d + 1)
        plus = img[cy + v, cx - d:cx + d + 1]
        minus = img[cy - v, cx - d:cx + d + 1]
        m01 += v * int((plus - minus).sum())
        m10 += int((u * (plus + minus)).sum())
    return fast_atan2_np(np.array([m01], F32), np.array([m10], F32))[0]


def describe_np(blurred, x, y, angle, pat):
    cy, cx = int(np.rint(F32(y))) + EDGE, int(np.rint(F32(x))) + EDGE
    factor = F32(np.pi / F32(180.0))                       # (float)(CV_PI / 180.f)
    ang = F32(F32(angle) * factor)
    a = F32(np.cos(np.float64(ang)))                       # correctly rounded float cos / sin
    b = F32(np.sin(np.float64(ang)))

    def value(px, py):
        px, py = F32(px), F32(py)
        dy = int(np.rint(F32(F32(px * b) + F32(py * a))))
        dx = int(np.rint(F32(F32(px * a) - F32(py * b))))
        return int(blurred[cy + dy, cx + dx])

    out = np.zeros(32, np.uint8)
    for i in range(32):
        val = 0
        for k in range(8):
            x1, y1, x2, y2 = pat[8 * i + k]
            val |= int(value(x1, y1) < value(x2, y2)) << k
        out[i] = val
    return out


@pytest.mark.parametrize("kind,w,h,n,seed", [("texture", 640, 480, 1000, 2000), ("noise", 333, 251, 500, 4),
                                              ("texture", 160, 120, 200, 9)])
def test_orientation_and_descriptor_match_oracle(kind, w, h, n, seed):
    img = synth.texture_frame(w, h, seed) if kind == "texture" else synth.noise_frame(w, h, seed)
    ex = RefExtractor(n)
    kps, desc = ex(img)
    pat, umax = pattern(), umax_np()
    assert np.array_equal(umax, ex.umax()[:HP + 1])
    at = 0
    checked = 0
    for lvl in range(8):
        lk = ex.level_keys(lvl)
        raw, blurred = ex.level(lvl), ex.level(lvl, blurred=True)
        # the level's keypoints are the output's next block, in the same order
        assert np.array_equal(kps["octave"][at:at + len(lk)], np.full(len(lk), lvl))
        step = max(1, len(lk) // 60)   # a spread sample per level keeps the test fast
        for k in range(0, len(lk), step):
            x, y, ang = lk["x"][k], lk["y"][k], lk["angle"][k]
            assert ic_angle_np(raw, x, y, umax) == ang, (lvl, k)
            assert np.array_equal(describe_np(blurred, x, y, ang, pat), desc[at + k]), (lvl, k)
            assert kps["angle"][at + k] == ang
            checked += 1
        at += len(lk)
    assert at == len(kps) and checked > 100
