"""Second, independent restatements of the OpenCV 2.4 internals the oracle
reproduces (VERDICT r03 "What's weak" 1, "Next" 8).

The oracle (oracle/ref_extract.cpp, oracle/ref_math.cpp) restates in C++
the OpenCV 2.4 routines ORBextractor calls; the product is checked against
it bit for bit.  These numpy float32 / integer restatements are written from
OpenCV 2.4's published algorithms, not from the oracle's code, so a slip in
either shows up as a mismatch here:

* cv::fastAtan2 (core/src/mathfuncs.cpp; IC_Angle, src/ORBextractor.cc:150):
  float32 polynomial in c = min/(max + (float)DBL_EPSILON), constants the
  float products of the static initialisers, octant fix-ups 90 - a, 180 - a,
  360 - a -- bit for bit on >= 10^5 integer moment pairs and the octant
  boundaries.
* cv::resize INTER_LINEAR 8U (imgproc/src/imgwarp.cpp; ComputePyramid,
  src/ORBextractor.cc:800): coefficient tables, the horizontal int pass, the
  SSE2 vertical pass (VResizeLinearVec_32s8u) and the scalar tail -- every
  level of the pyramid, with the REFLECT_101 borders of copyMakeBorder
  (src/ORBextractor.cc:806, :814).
* GaussianBlur 7x7 sigma 2 8U (imgproc/src/filter.cpp, smooth.cpp;
  src/ORBextractor.cc:760): the int kernel (float Gaussian x 256), exact row
  sums, the SSE2 float column pass (SymmColumnVec_32s8u) and its scalar tail
  -- every blurred level.
"""
import numpy as np
import pytest

from orb_slam_amd import synth
from oracle_lib import RefExtractor, load

F32 = np.float32


# ------------------------------------------------------------- fastAtan2
_PI180 = F32(180.0 / np.pi)            # (float)(180/CV_PI)
P1 = F32(F32(0.9997878412794807) * _PI180)
P3 = F32(F32(-0.3258083974640975) * _PI180)
P5 = F32(F32(0.1555786518463281) * _PI180)
P7 = F32(F32(-0.04432655554792128) * _PI180)
EPS = F32(np.finfo(np.float64).eps)    # (float)DBL_EPSILON


def fast_atan2_np(y, x):
    """OpenCV 2.4 cv::fastAtan2(y, x) in degrees, vectorised, every
    operation rounded to float32 as the scalar C++ evaluates it (no FMA)."""
    y = np.asarray(y, F32)
    x = np.asarray(x, F32)
    ax, ay = np.abs(x), np.abs(y)
    first = ax >= ay
    num = np.where(first, ay, ax)
    den = np.where(first, ax, ay)
    c = (num / (den + EPS)).astype(F32)
    c2 = (c * c).astype(F32)
    p = (((P7 * c2 + P5).astype(F32) * c2 + P3).astype(F32) * c2 + P1).astype(F32)
    a = (p * c).astype(F32)
    a = np.where(first, a, (F32(90.0) - a).astype(F32))
    a = np.where(x < 0, (F32(180.0) - a).astype(F32), a)
    a = np.where(y < 0, (F32(360.0) - a).astype(F32), a)
    return a.astype(F32)


def _oracle_atan2(ys, xs):
    L = load()
    return np.array([L.orbx_ref_fast_atan2(float(y), float(x)) for y, x in zip(ys, xs)], F32)


def test_fast_atan2_bitwise_random_moments():
    """10^5 integer moment pairs of IC_Angle's range (|m| <= 1.5e6: 700
    patch pixels x 15 x 255), bit for bit."""
    r = np.random.default_rng(2024)
    ys = r.integers(-1_500_000, 1_500_001, 100_000).astype(F32)
    xs = r.integers(-1_500_000, 1_500_001, 100_000).astype(F32)
    # small moments too (flat patches), where c is coarse
    ys[:20_000] = r.integers(-300, 301, 20_000)
    xs[:20_000] = r.integers(-300, 301, 20_000)
    got, want = fast_atan2_np(ys, xs), _oracle_atan2(ys, xs)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), int((got != want).sum())


def test_fast_atan2_bitwise_octant_boundaries():
    """x = +-y, x = 0, y = 0, and the pairs one step off the diagonals, in
    all four quadrants, bit for bit."""
    v = np.concatenate([np.arange(0, 2000), r_big := np.array([2 ** k for k in range(11, 21)]), r_big + 1])
    ys, xs = [], []
    for a in v:
        for d in (-1, 0, 1):
            for sy in (1, -1):
                for sx in (1, -1):
                    ys += [sy * a, sy * a, 0, sy * a]
                    xs += [sx * (a + d), 0, sx * a, sx * a]
    ys, xs = np.array(ys, F32), np.array(xs, F32)
    got, want = fast_atan2_np(ys, xs), _oracle_atan2(ys, xs)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), int((got != want).sum())
    assert np.all((got >= 0) & (got <= 360))


# ------------------------------------------------------------- cv::resize
def _reflect101(p, n):
    p = np.asarray(p)
    if n == 1:
        return np.zeros_like(p)
    period = 2 * n - 2
    p = np.abs(p) % period
    return np.where(p >= n, period - p, p)


def _coef_tables(dst_n, src_n):
    """cv::resize's per-axis tables for INTER_LINEAR with fixed point
    (INTER_RESIZE_COEF_SCALE 2048): source index, two int16 weights, and
    xmax (the first column whose right tap would fall outside)."""
    scale = float(src_n) / float(dst_n)
    d = np.arange(dst_n, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(F32)         # (float)((dx + 0.5) * scale_x - 0.5)
    s = np.floor(f).astype(np.int64)                  # cvFloor
    f = (f - s.astype(F32)).astype(F32)
    lo = s < 0
    f[lo], s[lo] = F32(0), 0
    over = s + 1 >= src_n
    xmax = int(np.argmax(over)) if over.any() else dst_n
    clamp = s >= src_n - 1
    f[clamp], s[clamp] = F32(0), src_n - 1
    w0 = np.rint((F32(1) - f).astype(F32) * F32(2048)).astype(np.int64)   # saturate_cast<short>(c * 2048)
    w1 = np.rint(f * F32(2048)).astype(np.int64)
    return s, w0, w1, xmax


def _vec_cols(width, strict4):
    """Columns an SSE2 16-wide loop followed by a 4-wide loop covers
    (VResizeLinearVec_32s8u: x < w - 4; SymmColumnVec_32s8u: x <= w - 4)."""
    x = 0
    while x <= width - 16:
        x += 16
    while (x < width - 4) if strict4 else (x <= width - 4):
        x += 4
    return x


def _sat16(v):
    return np.clip(v, -32768, 32767)


def resize_linear_np(src, dw, dh):
    """cv::resize(src, dst, Size(dw, dh), 0, 0, INTER_LINEAR) for CV_8UC1."""
    sh, sw = src.shape
    src = src.astype(np.int64)
    if sw == 2 * dw and sh == 2 * dh:   # exact 2x: INTER_AREA's fast path
        s = src[0::2, 0::2] + src[0::2, 1::2] + src[1::2, 0::2] + src[1::2, 1::2]
        return ((s + 2) >> 2).astype(np.uint8)
    xs, a0, a1, xmax = _coef_tables(dw, sw)
    # the row table keeps unclamped indices and weights; rows are clipped
    # when fetched
    f = ((np.arange(dh) + 0.5) * (float(sh) / dh) - 0.5).astype(F32)
    ys = np.floor(f).astype(np.int64)
    fy = (f - ys.astype(F32)).astype(F32)
    b0 = np.rint((F32(1) - fy).astype(F32) * F32(2048)).astype(np.int64)
    b1 = np.rint(fy * F32(2048)).astype(np.int64)

    def hpass(rows):
        out = rows[:, xs] * a0 + np.where(np.arange(dw) < xmax, rows[:, np.minimum(xs + 1, sw - 1)] * a1, 0)
        out[:, xmax:] = rows[:, xs[xmax:]] * 2048
        return out

    r0 = hpass(src[np.clip(ys, 0, sh - 1)])
    r1 = hpass(src[np.clip(ys + 1, 0, sh - 1)])
    nvec = _vec_cols(dw, True)
    B0, B1 = b0[:, None], b1[:, None]
    # SSE2: (S >> 4) packed to int16, mulhi with beta, saturating adds, + 2, >> 2
    m0 = (_sat16(r0 >> 4) * B0) >> 16
    m1 = (_sat16(r1 >> 4) * B1) >> 16
    vec = _sat16(_sat16(m0 + m1) + 2) >> 2
    tail = (r0 * B0 + r1 * B1 + (1 << 21)) >> 22
    out = np.where(np.arange(dw)[None, :] < nvec, vec, tail)
    return np.clip(out, 0, 255).astype(np.uint8)


def level_sizes(w, h, nlevels, scale):
    inv = F32(1.0 / np.float64(F32(scale)))     # mvInvScaleFactor: 1 / scaleFactor, accumulated in float
    s, out = F32(1.0), []
    for _ in range(nlevels):
        out.append((int(np.rint(F32(w) * s)), int(np.rint(F32(h) * s))))
        s = F32(s * inv)
    return out


def pyramid_np(img, nlevels=8, scale=1.2):
    """ComputePyramid (src/ORBextractor.cc:781-822): padded (w + 32) x
    (h + 32) levels, level 0 the image with a REFLECT_101 border, level l the
    resize of level l - 1's ROI with its own REFLECT_101 border."""
    E = 16
    out = []
    prev = None
    for (w, h) in level_sizes(img.shape[1], img.shape[0], nlevels, scale):
        roi = img if prev is None else resize_linear_np(prev, w, h)
        yy = _reflect101(np.arange(-E, h + E), h)
        xx = _reflect101(np.arange(-E, w + E), w)
        out.append(roi[yy][:, xx])
        prev = roi
    return out


# ----------------------------------------------------------- GaussianBlur
def gaussian_int_kernel():
    """getGaussianKernel(7, 2, CV_32F), then convertTo(CV_32S, 256) for the
    8U fixed-point smoothing path."""
    x = np.arange(7, dtype=np.float64) - 3.0
    cf = np.exp((-0.5 / 4.0) * x * x).astype(F32)
    total = np.float64(cf.astype(np.float64).sum())
    cf = (cf.astype(np.float64) * (1.0 / total)).astype(F32)
    return np.rint(cf * F32(256.0)).astype(np.int64)


def blur_np(padded, w, h):
    """GaussianBlur 7x7 in place on the ROI of a padded level: the parent's
    border pixels feed the filter and stay unblurred."""
    k = gaussian_int_kernel()
    E = 16
    P = padded.astype(np.int64)
    rows = sum(k[i] * P[E - 3:E + h + 3, E + i - 3:E + i - 3 + w] for i in range(7))   # rows -3 .. h+2
    ky = (k[3:].astype(np.float64) * (1.0 / 65536)).astype(F32)
    s = rows[3:3 + h].astype(F32) * ky[0] + F32(0)
    for j in range(1, 4):
        s = (s + (rows[3 + j:3 + j + h] + rows[3 - j:3 - j + h]).astype(F32) * ky[j]).astype(F32)
    vec = np.clip(np.rint(s).astype(np.int64), -32768, 32767)
    t = k[3] * rows[3:3 + h]
    for j in range(1, 4):
        t = t + k[3 + j] * (rows[3 + j:3 + j + h] + rows[3 - j:3 - j + h])
    tail = (t + (1 << 15)) >> 16
    nvec = _vec_cols(w, False)
    roi = np.clip(np.where(np.arange(w)[None, :] < nvec, vec, tail), 0, 255).astype(np.uint8)
    out = padded.copy()
    out[E:E + h, E:E + w] = roi
    return out


def test_gaussian_int_kernel():
    """The rounded taps are {18, 34, 49, 55, 49, 34, 18}: they sum to 257,
    not 256, so a bright enough column saturates."""
    k = gaussian_int_kernel()
    assert list(k) == [18, 34, 49, 55, 49, 34, 18] and k.sum() == 257


@pytest.mark.parametrize("w,h,seed,kind", [(640, 480, 2000, "texture"), (97, 71, 3, "texture"),
                                           (160, 120, 5, "noise"), (333, 250, 7, "texture")])
def test_pyramid_and_blur_match_oracle(w, h, seed, kind):
    """Every raw and blurred pyramid level of an oracle extraction equals the
    numpy restatement, byte for byte."""
    img = synth.texture_frame(w, h, seed) if kind == "texture" else synth.noise_frame(w, h, seed)
    ex = RefExtractor(1000)
    ex(img)
    sizes = level_sizes(w, h, 8, 1.2)
    for l, P in enumerate(pyramid_np(img)):
        raw = ex.level(l)
        assert raw.shape == P.shape and np.array_equal(raw, P), ("raw", l)
        lw, lh = sizes[l]
        assert np.array_equal(ex.level(l, blurred=True), blur_np(raw, lw, lh)), ("blurred", l)


@pytest.mark.parametrize("sw,sh,dw,dh", [(64, 48, 53, 40), (40, 40, 20, 20), (31, 17, 26, 14), (200, 9, 167, 8),
                                         (21, 21, 40, 40)])
def test_resize_matches_oracle(sw, sh, dw, dh):
    """cv::resize restatement against orbx_ref_resize on odd ratios, the
    exact 2x (INTER_AREA fast path) and an upscale."""
    import ctypes
    src = np.random.default_rng(sw * 100 + dw).integers(0, 256, (sh, sw), dtype=np.uint8)
    dst = np.zeros((dh, dw), np.uint8)
    L = load()
    assert L.orbx_ref_resize(src.ctypes.data_as(ctypes.c_void_p), sw, sw, sh, dst.ctypes.data_as(ctypes.c_void_p),
                             dw, dw, dh) == 0
    assert np.array_equal(resize_linear_np(src, dw, dh), dst)


@pytest.mark.gpu
def test_product_pyramid_matches_numpy():
    """The device pyramid (raw and blurred) against the numpy restatement
    directly, without the oracle in between."""
    import orb_slam_amd as ox
    img = synth.texture_frame(640, 480, 2000)
    ctx = ox.Context(nfeatures=1000, max_w=640, max_h=480, slots=1)
    try:
        ctx.upload(img)
        ctx.extract(0, 1)
        ctx.sync()
        sizes = level_sizes(640, 480, 8, 1.2)
        for l, P in enumerate(pyramid_np(img)):
            lw, lh = sizes[l]
            assert np.array_equal(ctx.level(0, l), P), ("raw", l)
            assert np.array_equal(ctx.level(0, l, blurred=True), blur_np(P, lw, lh)), ("blurred", l)
    finally:
        ctx.close()
