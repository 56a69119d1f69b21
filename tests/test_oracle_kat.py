"""Known-answer tests for the CPU restatement (oracle/), run without a GPU.

The reference ships no tests or fixtures for this path (SURVEY.md section
8c: "parity unpinned"), so the oracle is pinned here by values that follow
from the reference's own source and its dependencies' published semantics:

* fastAtan2 exact quadrant values and its documented ~0.3 deg accuracy
  (OpenCV 2.4 mathfuncs.cpp; IC_Angle src/ORBextractor.cc:124-151 returns
  fastAtan2 at :150);
* DescriptorDistance popcount identity (src/ORBmatcher.cc:1794-1810);
* a hand-built FAST-9 patch whose score is known in closed form
  (cv::FAST with nonmax suppression, called per cell at
  src/ORBextractor.cc:607 and, for <= 3 corners, :613);
* cosf / sinf of the descriptor angle (computeOrbDescriptor,
  src/ORBextractor.cc:159-160) against correctly rounded values;
* umax, features per level, level sizes (src/ORBextractor.cc:457-511:
  scale factors :462-471, quotas :476-487, umax :495-510);
* retainBest keeps exactly the top-n responses (src/ORBextractor.cc:683-685,
  :697-701);
* SE3 exponential against scipy's matrix exponential, and the analytic
  EdgeSE3ProjectXYZ Jacobians against central finite differences
  (Thirdparty/g2o/g2o/types/sba/types_six_dof_expmap.cpp:384-420);
* a noise-free local BA recovers the ground truth (src/Optimizer.cc:449-535).

The product's own host tables (orbx_describe_levels) are checked against
the oracle here too: that call needs no device.
"""
import ctypes

import numpy as np
import pytest
import scipy.linalg

import orb_slam_amd as ox
from orb_slam_amd import synth, synth_ba as sb
from oracle_lib import KEYPOINT, RefExtractor, load, ptr


def _d(*a):
    return np.ascontiguousarray(np.array(a, np.float64).ravel())


# ---------------------------------------------------------------- angles
@pytest.mark.parametrize("y,x,want", [(0.0, 1.0, 0.0), (1.0, 0.0, 90.0), (0.0, -1.0, 180.0),
                                      (-1.0, 0.0, 270.0), (0.0, 0.0, 0.0), (5.0, 5.0, 45.0)])
def test_fast_atan2_quadrants(ref, y, x, want):
    assert abs(ref.orbx_ref_fast_atan2(y, x) - want) < 0.3


def test_fast_atan2_accuracy(ref):
    r = np.random.default_rng(0)
    for y, x in r.integers(-3000, 3000, size=(2000, 2)).astype(np.float32):
        a = ref.orbx_ref_fast_atan2(float(y), float(x))
        assert 0.0 <= a < 360.0
        want = np.degrees(np.arctan2(y, x)) % 360.0
        d = abs(a - want)
        assert min(d, 360 - d) < 0.3


def test_sincos_is_correctly_rounded_float(ref):
    """computeOrbDescriptor's cos/sin (src/ORBextractor.cc:159-160) are evaluated as the
    correctly rounded float of the true value (see oracle/ref_math.cpp)."""
    r = np.random.default_rng(1)
    for a in r.uniform(0, 2 * np.pi, 3000).astype(np.float32):
        c = np.float32(ref.orbx_ref_cosf(float(a)))
        s = np.float32(ref.orbx_ref_sinf(float(a)))
        for got, exact in ((c, np.cos(np.float64(a))), (s, np.sin(np.float64(a)))):
            lo, hi = np.nextafter(got, np.float32(-2)), np.nextafter(got, np.float32(2))
            # exact lies within half an ulp of got
            assert abs(exact - np.float64(got)) <= 0.5 * (np.float64(hi) - np.float64(lo)) / 2 + 1e-30


# ---------------------------------------------------------------- distance
def test_descriptor_distance_popcount(ref):
    r = np.random.default_rng(2)
    for _ in range(200):
        a = r.integers(0, 256, 32, dtype=np.uint8)
        b = r.integers(0, 256, 32, dtype=np.uint8)
        want = int(np.unpackbits(a ^ b).sum())
        assert ref.orbx_ref_descriptor_distance(ptr(a), ptr(b)) == want
        assert ox.lib().orbx_descriptor_distance(ptr(a), ptr(b)) == want
    z = np.zeros(32, np.uint8)
    assert ref.orbx_ref_descriptor_distance(ptr(z), ptr(z)) == 0
    assert ref.orbx_ref_descriptor_distance(ptr(z), ptr(np.full(32, 255, np.uint8))) == 256


# ---------------------------------------------------------------- FAST
def _fast(ref, img, th):
    img = np.ascontiguousarray(img, np.uint8)
    out = np.zeros(4096, KEYPOINT)
    n = ctypes.c_int()
    assert ref.orbx_ref_fast_cell(ptr(img), img.shape[1], img.shape[0], img.shape[1], th, ptr(out), out.size,
                                  ctypes.byref(n)) == 0
    return out[:n.value]


def test_fast_single_bright_pixel(ref):
    img = np.full((16, 16), 50, np.uint8)
    img[8, 8] = 200
    k = _fast(ref, img, 20)
    assert len(k) == 1
    assert (k[0]["x"], k[0]["y"]) == (8.0, 8.0)
    # all 16 circle pixels are 150 darker: the largest threshold that still
    # passes the strict test is 149 (cv::FAST score semantics)
    assert k[0]["response"] == 149.0
    assert len(_fast(ref, img, 149)) == 1
    assert len(_fast(ref, img, 150)) == 0


def test_fast_flat_and_arc_lengths(ref):
    assert len(_fast(ref, np.full((32, 32), 90, np.uint8), 5)) == 0
    # an arc of exactly 8 contiguous darker circle pixels is not a corner,
    # 9 is (FAST-9/16)
    circle = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
              (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]
    for arc, corner in ((8, False), (9, True), (12, True)):
        img = np.full((15, 15), 100, np.uint8)
        for dx, dy in circle[:arc]:
            img[7 + dy, 7 + dx] = 10
        ks = _fast(ref, img, 20)
        at_center = [k for k in ks if (k["x"], k["y"]) == (7.0, 7.0)]
        assert bool(at_center) == corner, arc
        if corner:
            assert at_center[0]["response"] == 89.0


# ---------------------------------------------------------------- geometry
def test_umax_table():
    assert list(RefExtractor().umax()) == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]


def test_features_per_level():
    want = [217, 181, 151, 126, 105, 87, 73, 60]
    assert list(RefExtractor(1000, 1.2, 8).features_per_level()) == want
    assert sum(RefExtractor(2000, 1.2, 8).features_per_level()) == 2000
    assert [l["n_desired"] for l in ox.describe_levels(640, 480)] == want


def test_scale_factors(ref):
    e = RefExtractor(1000, 1.2, 8)
    s = np.zeros(8, np.float32)
    inv = np.zeros(8, np.float32)
    assert ref.orbx_ref_scale_factors(e.h, ptr(s), ptr(inv), 8) == 8
    assert s[0] == 1.0 and abs(s[7] - 1.2 ** 7) < 1e-5
    assert np.allclose(s * inv, 1.0, atol=1e-6)


@pytest.mark.parametrize("w,h,nf", [(640, 480, 1000), (1920, 1080, 2000), (333, 251, 500), (96, 80, 100)])
def test_level_sizes_product_vs_oracle(w, h, nf):
    e = RefExtractor(nf, 1.2, 8)
    e(synth.texture_frame(w, h, 0))
    prod = ox.describe_levels(w, h, nf)
    for l in range(8):
        # oracle levels carry the EDGE_THRESHOLD=16 border (src/ORBextractor.cc:787)
        assert e.level(l).shape == (prod[l]["h"] + 32, prod[l]["w"] + 32), l
        assert prod[l]["n_desired"] == e.features_per_level()[l]
    if (w, h) == (640, 480):
        assert [(p["w"], p["h"]) for p in prod] == [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231),
                                                    (257, 193), (214, 161), (179, 134)]


def test_describe_levels_rejects_bad_args():
    with pytest.raises(ox.OrbxError):
        ox.describe_levels(640, 480, nfeatures=0)
    with pytest.raises(ox.OrbxError):
        ox.describe_levels(640, 480, scale_factor=1.0)


# ---------------------------------------------------------------- resize / retain
def test_resize_constant_and_identity(ref):
    src = np.full((100, 120), 77, np.uint8)
    dst = np.zeros((83, 100), np.uint8)
    assert ref.orbx_ref_resize(ptr(src), 120, 120, 100, ptr(dst), 100, 100, 83) == 0
    assert (dst == 77).all()
    r = np.random.default_rng(3).integers(0, 256, (40, 50), dtype=np.uint8)
    same = np.zeros_like(r)
    assert ref.orbx_ref_resize(ptr(r), 50, 50, 40, ptr(same), 50, 50, 40) == 0
    assert np.array_equal(same, r)


def test_resize_exact_half_is_area_fast(ref):
    """Exactly 2x: cv::resize reroutes INTER_LINEAR to INTER_AREA's fast path,
    (S00 + S01 + S10 + S11 + 2) >> 2 (ResizeAreaFastVec<uchar>); a ratio just
    off 2 stays INTER_LINEAR."""
    r = np.random.default_rng(4).integers(0, 256, (48, 64), dtype=np.uint8)
    dst = np.zeros((24, 32), np.uint8)
    assert ref.orbx_ref_resize(ptr(r), 64, 64, 48, ptr(dst), 32, 32, 24) == 0
    s = r.astype(np.int32)
    want = (s[0::2, 0::2] + s[0::2, 1::2] + s[1::2, 0::2] + s[1::2, 1::2] + 2) >> 2
    assert np.array_equal(dst, want)
    odd = np.zeros((24, 33), np.uint8)   # 64 -> 33 columns: linear
    assert ref.orbx_ref_resize(ptr(r), 64, 64, 48, ptr(odd), 33, 33, 24) == 0


@pytest.mark.parametrize("n,keep,seed", [(50, 10, 0), (200, 37, 1), (1000, 217, 2), (30, 30, 3), (30, 40, 4),
                                         (500, 1, 5)])
def test_retain_best_keeps_top_n(ref, n, keep, seed):
    r = np.random.default_rng(seed)
    resp = r.integers(0, 40, n).astype(np.float32)        # many ties, like FAST scores
    out = np.zeros(n, np.int32)
    m = ref.orbx_ref_retain_best(ptr(resp), n, keep, ptr(out))
    assert m == min(n, keep)
    kept = np.sort(resp[out[:m]])[::-1]
    assert np.array_equal(kept, np.sort(resp)[::-1][:m])
    assert len(set(out[:m].tolist())) == m


# ---------------------------------------------------------------- SE3 / edge
def _q2R(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def _hat(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])


def _se3_exp(ref, u):
    q = np.zeros(4)
    t = np.zeros(3)
    ref.orbx_ref_se3_exp.argtypes = [ctypes.c_void_p] * 3
    ref.orbx_ref_se3_exp(ptr(_d(u)), ptr(q), ptr(t))
    return q, t


@pytest.mark.parametrize("seed", range(5))
def test_se3_exp_matches_matrix_exponential(ref, seed):
    u = np.random.default_rng(seed).normal(0, 0.4, 6)
    q, t = _se3_exp(ref, u)
    twist = np.zeros((4, 4))
    twist[:3, :3] = _hat(u[:3])      # g2o update order: omega, then upsilon
    twist[:3, 3] = u[3:]
    E = scipy.linalg.expm(twist)
    assert abs(np.linalg.norm(q) - 1) < 1e-12
    assert np.allclose(_q2R(q), E[:3, :3], atol=1e-12)
    assert np.allclose(t, E[:3, 3], atol=1e-12)


def _edge(ref, pose, X, cam, obs):
    err = np.zeros(2)
    A = np.zeros(6)
    B = np.zeros(12)
    ref.orbx_ref_edge_linearize.argtypes = [ctypes.c_void_p] * 7
    ref.orbx_ref_edge_linearize(ptr(_d(pose)), ptr(_d(X)), ptr(_d(cam)), ptr(_d(obs)), ptr(err), ptr(A), ptr(B))
    return err, A.reshape(2, 3), B.reshape(2, 6)


@pytest.mark.parametrize("seed", range(6))
def test_edge_jacobians_match_finite_differences(ref, seed):
    r = np.random.default_rng(seed)
    q = r.normal(size=4)
    q /= np.linalg.norm(q)
    t = r.normal(0, 0.5, 3)
    R = _q2R(q)
    X = R.T @ (np.array([r.uniform(-1, 1), r.uniform(-1, 1), r.uniform(2, 5)]) - t)   # in front of camera
    cam = [520.0, 510.0, 320.0, 240.0]
    obs = [300.0, 250.0]
    pose = np.concatenate([q, t])
    err, A, B = _edge(ref, pose, X, cam, obs)

    def error_at(Rm, tm, Xw):
        pc = Rm @ Xw + tm
        return np.array(obs) - np.array([cam[0] * pc[0] / pc[2] + cam[2], cam[1] * pc[1] / pc[2] + cam[3]])

    assert np.allclose(err, error_at(R, t, X), atol=1e-9)
    h = 1e-6
    for k in range(3):
        d = np.zeros(3)
        d[k] = h
        fd = (error_at(R, t, X + d) - error_at(R, t, X - d)) / (2 * h)
        assert np.allclose(A[:, k], fd, rtol=1e-5, atol=1e-4), k
    for k in range(6):
        d = np.zeros(6)
        d[k] = h
        cols = []
        for s in (1, -1):
            dq, dt = _se3_exp(ref, s * d)
            dR = _q2R(dq)
            cols.append(error_at(dR @ R, dR @ t + dt, X))         # T <- exp(d) * T (g2o oplus)
        fd = (cols[0] - cols[1]) / (2 * h)
        assert np.allclose(B[:, k], fd, rtol=1e-5, atol=1e-4), k


# ---------------------------------------------------------------- local BA
def test_noise_free_ba_recovers_ground_truth(ref):
    prob = sb.make_problem(n_kf=6, n_points=300, seed=11, outlier_frac=0.0, pix_noise=0.0, point_noise=0.01)
    p, arrs = sb.to_ctypes(prob)
    es = np.zeros(p.n_edges, np.uint8)
    pb = np.zeros(p.n_points, np.uint8)
    st = sb.BAStats()
    ref.orbx_ref_lba.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p]
    assert ref.orbx_ref_lba(ctypes.byref(p), 5, 10, ptr(es), ptr(pb), ctypes.byref(st)) == 0
    assert st.chi2_initial[0] > 1.0
    assert st.chi2_final[1] < 1e-6 * st.chi2_initial[0] + 1e-4
    assert not es.any() and not pb.any()
    for k, (Rt, tt) in enumerate(prob["poses_true"]):
        assert np.allclose(_q2R(arrs["pose_q"][k]), Rt, atol=2e-5), k
        assert np.allclose(arrs["pose_t"][k], tt, atol=2e-5), k
    assert np.abs(arrs["points"] - prob["points_true"]).max() < 1e-3
