"""GPU parity of ORB extraction against the CPU restatement (oracle).

Every comparison is bit-exact: pyramid levels (raw and blurred), keypoints
(all seven cv::KeyPoint fields, in reference order) and descriptors.
Reference: ORBextractor::operator() (src/ORBextractor.cc:718-779).
"""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
from orb_slam_amd import synth
from oracle_lib import KEYPOINT as KEYPOINT_DT, RefExtractor

pytestmark = pytest.mark.gpu

CASES = [
    ("texture", 640, 480, 1000, 1),
    ("noise", 640, 480, 1000, 2),
    ("flat", 640, 480, 1000, 0),
    ("texture", 96, 80, 100, 3),
    ("noise", 333, 251, 500, 4),
    ("texture", 1920, 1080, 2000, 5),
    ("noise", 1920, 1080, 2000, 7),      # cell lists beyond the LDS replay cap
    ("rects", 640, 480, 1000, 6),
]


def make(kind, w, h, seed):
    if kind == "texture":
        return synth.texture_frame(w, h, seed)
    if kind == "noise":
        return synth.noise_frame(w, h, seed)
    if kind == "flat":
        return synth.flat_frame(w, h)
    r = np.random.default_rng(seed)
    img = np.full((h, w), 40, np.uint8)
    for _ in range(60):
        x, y = r.integers(0, w - 8), r.integers(0, h - 8)
        img[y:y + r.integers(4, 60), x:x + r.integers(4, 60)] = r.integers(0, 256)
    return img


def assert_kps_equal(a, b):
    assert len(a) == len(b), (len(a), len(b))
    for f in ox.KEYPOINT.names:
        if not np.array_equal(a[f], b[f]):
            bad = np.nonzero(a[f] != b[f])[0]
            raise AssertionError(f"field {f}: {len(bad)} mismatches, first at {bad[0]}: "
                                 f"gpu={a[bad[0]]} ref={b[bad[0]]}")


@pytest.mark.parametrize("kind,w,h,n,seed", CASES)
def test_extract_matches_oracle(kind, w, h, n, seed):
    img = make(kind, w, h, seed)
    ref = RefExtractor(n)
    rk, rd = ref(img)
    ctx = ox.Context(nfeatures=n, max_w=w, max_h=h, slots=1)
    ctx.upload(img)
    ctx.extract(0, 1)
    ctx.sync()
    for lvl in range(8):
        g = ctx.level(0, lvl)
        r = ref.level(lvl)
        assert g.shape == r.shape
        assert np.array_equal(g, r), f"raw level {lvl}: {np.count_nonzero(g != r)} bytes differ"
        gb = ctx.level(0, lvl, blurred=True)
        rb = ref.level(lvl, blurred=True)
        assert np.array_equal(gb, rb), f"blurred level {lvl}: {np.count_nonzero(gb != rb)} bytes differ"
    gk, gd = ctx.features(0)
    assert_kps_equal(gk, rk)
    assert np.array_equal(gd, rd), f"{np.count_nonzero((gd != rd).any(1))} descriptors differ"
    ctx.close()


def test_operator_call_and_batch_consistency():
    w, h, n = 640, 480, 1000
    frames = synth.sequence(w, h, 6, seed=11)
    ref = RefExtractor(n)
    ctx = ox.Context(nfeatures=n, max_w=w, max_h=h, slots=6)
    # batched device-resident path
    ctx.upload(frames)
    ctx.extract(0, 6)
    ctx.sync()
    for s in range(6):
        gk, gd = ctx.features(s)
        rk, rd = ref(frames[s])
        assert_kps_equal(gk, rk)
        assert np.array_equal(gd, rd)
    # drop-in operator() form (host in / host out)
    k1, d1 = ctx(frames[2])
    rk, rd = ref(frames[2])
    assert_kps_equal(k1, rk)
    assert np.array_equal(d1, rd)
    # a mask does not change the result (the reference never reads the
    # cell mask, src/ORBextractor.cc:601-613)
    mask = np.zeros((h, w), np.uint8)
    mask[:, : w // 2] = 255
    km, dm = ctx(frames[2], mask)
    assert_kps_equal(km, rk)
    assert np.array_equal(dm, rd)
    # empty image: returns without keypoints (src/ORBextractor.cc:721-722)
    k0, d0 = ctx(np.zeros((0, 0), np.uint8))
    assert len(k0) == 0 and len(d0) == 0
    ctx.close()


def test_large_batch_paths_match_oracle():
    """A 64-frame batch (the bench's launch shape, many workgroups per
    launch): spot-check frames of the batch bit-exactly."""
    w, h, B = 640, 480, 64
    frames = synth.sequence(w, h, B, seed=99)
    ctx = ox.Context(nfeatures=1000, max_w=w, max_h=h, slots=B)
    ctx.upload(frames)
    ctx.extract(0, B)
    ctx.sync()
    ref = RefExtractor(1000)
    for s in (0, 17, 63):
        rk, rd = ref(frames[s])
        gk, gd = ctx.features(s)
        assert_kps_equal(gk, rk)
        assert np.array_equal(gd, rd)
        for lvl in (1, 4, 7):
            assert np.array_equal(ctx.level(s, lvl), ref.level(lvl)), (s, lvl)
    ctx.close()


@pytest.mark.parametrize("kind,w,h,n,seed", CASES)
def test_single_frame_cascade_pyramid_identical(kind, w, h, n, seed):
    """orbx_extract's single-frame graph builds the raw pyramid as one
    band-cascade launch (k_pyr_cascade, with FAST and the blur in one grid);
    the batch path uses the staged per-level launches.  Both leave
    byte-identical padded levels (raw and blurred) in slot 0 and the same
    keypoints and descriptors."""
    img = make(kind, w, h, seed)
    res = []
    for path in ("graph", "staged"):
        ctx = ox.Context(nfeatures=n, max_w=w, max_h=h, slots=1)
        if path == "graph":
            feats = ctx(img)
        else:
            ctx.upload(img[None])
            ctx.extract(0, 1)
            ctx.sync()
            feats = ctx.features(0)
        res.append([(ctx.level(0, lv), ctx.level(0, lv, blurred=True)) for lv in range(8)] + [feats])
        ctx.close()
    a, b = res
    for lv in range(8):
        assert np.array_equal(a[lv][0], b[lv][0]), f"raw level {lv}"
        assert np.array_equal(a[lv][1], b[lv][1]), f"blurred level {lv}"
    assert_kps_equal(a[8][0], b[8][0])
    assert np.array_equal(a[8][1], b[8][1])


@pytest.mark.parametrize("kind,w,h,n,seed", CASES)
def test_harris_score_matches_oracle(kind, w, h, n, seed):
    """scoreType == HARRIS_SCORE (src/ORBextractor.cc:616-620): the FAST
    corners are re-scored by HarrisResponses before both retainBest calls;
    keypoints (Harris responses included) and descriptors bit-exact."""
    img = make(kind, w, h, seed)
    ref = RefExtractor(n, score_type=0)
    rk, rd = ref(img)
    ctx = ox.Context(nfeatures=n, max_w=w, max_h=h, slots=1, score_type=0)
    ctx.upload(img)
    ctx.extract(0, 1)
    ctx.sync()
    gk, gd = ctx.features(0)
    assert_kps_equal(gk, rk)
    assert np.array_equal(gd, rd), f"{np.count_nonzero((gd != rd).any(1))} descriptors differ"
    ctx.close()


def test_harris_large_batch_pipeline():
    """HARRIS_SCORE through the multi-stream batch pipeline (64 frames in
    parts), spot-checked against the oracle."""
    w, h, B = 640, 480, 64
    frames = synth.sequence(w, h, B, seed=98)
    ctx = ox.Context(nfeatures=1000, max_w=w, max_h=h, slots=B, score_type=0)
    ctx.upload(frames)
    ctx.extract(0, B)
    ctx.sync()
    ref = RefExtractor(1000, score_type=0)
    for s in (0, 21, 42, 63):
        rk, rd = ref(frames[s])
        gk, gd = ctx.features(s)
        assert_kps_equal(gk, rk)
        assert np.array_equal(gd, rd)
    ctx.close()


# ORBextractor parameters other than Settings.yaml's defaults (nFeatures,
# scaleFactor, nLevels, fastTh: src/Tracking.cc:105-113); fastTh < 7 makes
# the threshold-7 fallback the higher threshold (src/ORBextractor.cc:607-614).
CONFIGS = [
    (500, 1.5, 4, 20, 1),
    (2000, 1.1, 12, 10, 1),
    (1200, 1.3, 6, 35, 1),
    (1000, 2.0, 3, 5, 1),
    (800, 1.25, 10, 20, 0),   # HARRIS_SCORE
]


@pytest.mark.parametrize("nf,scale,nlev,fth,score", CONFIGS)
@pytest.mark.parametrize("kind,w,h,seed", [("texture", 640, 480, 21), ("noise", 333, 251, 22)])
def test_extractor_configs_match_oracle(nf, scale, nlev, fth, score, kind, w, h, seed):
    img = make(kind, w, h, seed)
    ref = RefExtractor(nf, scale=scale, nlevels=nlev, fast_th=fth, score_type=score)
    rk, rd = ref(img)
    ctx = ox.Context(nfeatures=nf, scale_factor=scale, nlevels=nlev, score_type=score, fast_th=fth,
                     max_w=w, max_h=h, slots=1)
    assert ctx.GetLevels() == nlev
    ctx.upload(img)
    ctx.extract(0, 1)
    ctx.sync()
    for lvl in range(nlev):
        assert np.array_equal(ctx.level(0, lvl), ref.level(lvl)), f"raw level {lvl}"
        assert np.array_equal(ctx.level(0, lvl, blurred=True), ref.level(lvl, blurred=True)), f"blurred level {lvl}"
    gk, gd = ctx.features(0)
    assert_kps_equal(gk, rk)
    assert np.array_equal(gd, rd)
    ctx.close()


@pytest.mark.parametrize("nf,scale,nlev,fth,score", CONFIGS[:2])
def test_extractor_configs_batch_pipeline(nf, scale, nlev, fth, score):
    """A non-default configuration through the multi-stream batch path."""
    w, h, B = 640, 480, 64
    frames = synth.sequence(w, h, B, seed=31)
    ctx = ox.Context(nfeatures=nf, scale_factor=scale, nlevels=nlev, score_type=score, fast_th=fth,
                     max_w=w, max_h=h, slots=B)
    ctx.upload(frames)
    ctx.extract(0, B)
    ctx.sync()
    ref = RefExtractor(nf, scale=scale, nlevels=nlev, fast_th=fth, score_type=score)
    for s in (0, 33, 63):
        rk, rd = ref(frames[s])
        gk, gd = ctx.features(s)
        assert_kps_equal(gk, rk)
        assert np.array_equal(gd, rd)
    ctx.close()


@pytest.mark.parametrize("w,h", [(333, 251), (1000, 562)])
def test_ragged_large_batch_pipeline(w, h):
    """Frame widths that are not multiples of 16 (gathered level-0 border
    words, per-pixel resize tails) through the three-part batch pipeline."""
    B = 48
    frames = synth.sequence(w, h, B, seed=w)
    ctx = ox.Context(nfeatures=1000, max_w=w, max_h=h, slots=B)
    ctx.upload(frames)
    ctx.extract(0, B)
    ctx.sync()
    ref = RefExtractor(1000)
    for s in (0, 16, 47):
        rk, rd = ref(frames[s])
        gk, gd = ctx.features(s)
        assert_kps_equal(gk, rk)
        assert np.array_equal(gd, rd)
        assert np.array_equal(ctx.level(s, 3), ref.level(3))
    ctx.close()


def _random_configs(n, seed=2026):
    r = np.random.default_rng(seed)
    out = []
    for i in range(n):
        w, h = int(r.integers(48, 720)), int(r.integers(48, 560))
        out.append((w, h, int(r.integers(20, 2500)), float(np.float32(r.uniform(1.05, 1.6))), int(r.integers(1, 13)),
                    int(r.integers(1, 60)), int(r.integers(0, 2)), ("texture", "noise", "rects")[i % 3], i))
    return out


@pytest.mark.parametrize("w,h,nf,scale,nlev,fth,score,kind,seed", _random_configs(40))
def test_random_configs_match_oracle(w, h, nf, scale, nlev, fth, score, kind, seed):
    """Seeded random extractor configurations and frame sizes: where the
    oracle extracts, the GPU result is bit-exact; where the oracle refuses
    (a configuration the reference cannot run, e.g. an empty cell grid), the
    product refuses too."""
    img = make(kind, w, h, seed)
    ref = RefExtractor(nf, scale=scale, nlevels=nlev, fast_th=fth, score_type=score)
    kps = np.zeros(nf, KEYPOINT_DT)
    desc = np.zeros((nf, 32), np.uint8)
    n = ctypes.c_int()
    rc = ref.L.orbx_ref_extract(ref.h, img.ctypes.data_as(ctypes.c_void_p), w, h, w,
                                kps.ctypes.data_as(ctypes.c_void_p), desc.ctypes.data_as(ctypes.c_void_p), nf,
                                ctypes.byref(n))
    try:
        ctx = ox.Context(nfeatures=nf, scale_factor=scale, nlevels=nlev, score_type=score, fast_th=fth,
                         max_w=w, max_h=h, slots=1)
    except ox.OrbxError as e:
        assert rc != 0, f"product refused a configuration the oracle runs: {e}"
        return
    try:
        gk, gd = ctx(img)
    except ox.OrbxError as e:
        assert rc != 0, f"product refused a frame the oracle extracts: {e}"
        return
    finally:
        ctx.close()
    assert rc == 0, "product extracted a configuration the oracle refuses"
    rk, rd = kps[:n.value], desc[:n.value]
    assert_kps_equal(gk, rk)
    assert np.array_equal(gd, rd)


@pytest.mark.parametrize("w,h,nf,scale,nlev,fth,score,kind,seed", _random_configs(10, seed=77))
def test_random_configs_batch_pipeline(w, h, nf, scale, nlev, fth, score, kind, seed):
    """Random configurations through the multi-part batch pipeline (48
    frames: three parts), spot-checked against the oracle."""
    B = 48
    frames = synth.sequence(w, h, B, seed=seed + 500)
    ref = RefExtractor(nf, scale=scale, nlevels=nlev, fast_th=fth, score_type=score)
    try:
        ctx = ox.Context(nfeatures=nf, scale_factor=scale, nlevels=nlev, score_type=score, fast_th=fth,
                         max_w=w, max_h=h, slots=B)
    except ox.OrbxError:
        with pytest.raises(AssertionError):
            ref(frames[0])
        return
    ctx.upload(frames)
    ctx.extract(0, B)
    ctx.sync()
    for s in (0, 17, 47):
        rk, rd = ref(frames[s])
        gk, gd = ctx.features(s)
        assert_kps_equal(gk, rk)
        assert np.array_equal(gd, rd)
    ctx.close()


@pytest.mark.parametrize("w,h,nf,kind,fth", [
    (1920, 1080, 2000, "rects", 20),    # 336-pitch instance, three row bands per level-0 cell, flat cells fall back
    (1920, 1080, 2000, "noise", 20),    # dense corners in every band
    (1280, 1600, 400, "texture", 20),   # few huge cells: runtime-pitch instance, many bands
    (1280, 1600, 400, "rects", 45),     # ... with the threshold-7 fallback band by band
])
def test_row_bands_match_oracle(w, h, nf, kind, fth):
    """Tall FAST cells are scored in row bands (each window = band + 8 halo
    rows) so a workgroup's LDS stays small; corners, scores and their raster
    order must equal the whole-cell oracle, including cells whose <= 3
    corners at fastTh send every band back for the FAST(7) pass."""
    img = make(kind, w, h, 3)
    ctx = ox.Context(nfeatures=nf, fast_th=fth, max_w=w, max_h=h, slots=1)
    gk, gd = ctx(img)
    ctx.close()
    rk, rd = RefExtractor(nf, fast_th=fth)(img)
    assert_kps_equal(gk, rk)
    assert np.array_equal(gd, rd)
