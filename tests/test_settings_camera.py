"""The reference's own shipped configuration (Data/Settings.yaml:6-16, 27-40):
fx 268.9633, fy 269.9858, cx 157.6087, cy 114.6369, k1 -0.4157, k2 0.2624,
p1 = p2 = 0, k3 -0.1178 on a 320 x 240 frame, nFeatures 1000, scaleFactor
1.2, nLevels 8, fastTh 20, FAST score -- the only input data the reference
holds for this path.

Frame construction with that camera (src/Frame.cc:40-130): extraction, then
UndistortKeyPoints (:288-318; cv::undistortPoints with the five
coefficients), ComputeImageBounds (:320-348; the strongly barrel-distorted
corners put the bounds well outside 0..320 x 0..240), the 64 x 48 grid on
those bounds (:76-77, :108-122), then SearchForInitialization between two
frames (src/ORBmatcher.cc:598-713) and a motion-model SearchByProjection
(:1507-1620).  CPU tests pin the oracle's undistortion against a numpy
forward model and the host bounds against the oracle; GPU tests require the
device path (host-pointer and slot-resident forms) to equal the oracle bit
for bit.
"""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
from orb_slam_amd import synth
from oracle_lib import RefExtractor, load, ptr

W, H = 320, 240
K = np.array([268.9633, 269.9858, 157.6087, 114.6369], np.float32)   # Data/Settings.yaml:6-9
DIST = np.array([-0.4157, 0.2624, 0.0, 0.0, -0.1178], np.float32)     # k1 k2 p1 p2 k3 (:12-16)


def ref_undistort(k):
    L = load()
    L.orbx_ref_undistort_keypoints.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4
    out = np.zeros_like(k)
    assert L.orbx_ref_undistort_keypoints(len(k), ptr(k), ptr(K), ptr(DIST), ptr(out)) == 0
    return out


def ref_bounds():
    L = load()
    L.orbx_ref_compute_image_bounds.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 3
    b = np.zeros(4, np.float32)
    assert L.orbx_ref_compute_image_bounds(W, H, ptr(K), ptr(DIST), ptr(b)) == 0
    return b


def view(k, d, b):
    v = ox.frame_view(k, d, W, H)
    v.min_x, v.max_x, v.min_y, v.max_y = (float(x) for x in b)
    return v


def forward(xu, yu):
    """Brown-Conrady distortion of normalised coordinates (the model
    cv::undistortPoints inverts)."""
    k1, k2, p1, p2, k3 = (float(v) for v in DIST)
    r2 = xu * xu + yu * yu
    rad = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 ** 3
    return xu * rad + 2 * p1 * xu * yu + p2 * (r2 + 2 * xu * xu), yu * rad + p1 * (r2 + 2 * yu * yu) + 2 * p2 * xu * yu


def test_oracle_undistortion_inverts_settings_camera():
    """The oracle's iterative inversion, re-distorted by the forward model,
    lands back on the keypoints: cv::undistortPoints' fixed 5 iterations
    converge to 1e-3 px within 100 px of the principal point and 0.05 px
    within 150 px; at the corners, where this barrel distortion is
    strongest, 5 iterations leave ~1.5 px (the reference's own result)."""
    rng = np.random.default_rng(3)
    k = np.zeros(400, ox.KEYPOINT)
    k["x"], k["y"] = rng.uniform(0, W, 400), rng.uniform(0, H, 400)
    u = ref_undistort(k)
    xd, yd = forward((u["x"] - K[2]) / K[0], (u["y"] - K[3]) / K[1])
    px, py = xd * K[0] + K[2], yd * K[1] + K[3]
    err = np.hypot(px - k["x"], py - k["y"])
    r = np.hypot(k["x"] - K[2], k["y"] - K[3])
    assert err[r < 100].max() < 1e-3 and err[r < 150].max() < 0.05 and err.max() < 3.0


def test_image_bounds_settings_camera():
    """ComputeImageBounds of the shipped camera: product (host) == oracle,
    and the corners undistort outside the image on every side."""
    b = ref_bounds()
    g = np.zeros(4, np.float32)
    assert ox.lib().orbx_compute_image_bounds(W, H, ox._ptr(K), ox._ptr(DIST), ox._ptr(g)) == 0
    assert np.array_equal(g, b)
    assert b[0] < 0 and b[1] > W and b[2] < 0 and b[3] > H
    # the corners' own undistortion (src/Frame.cc:324-338) gives those bounds
    c = np.zeros(4, ox.KEYPOINT)
    c["x"], c["y"] = [0, W, 0, W], [0, 0, H, H]
    u = ref_undistort(c)
    assert b[0] == min(np.floor(u["x"][0]), np.floor(u["x"][2]))
    assert b[1] == max(np.ceil(u["x"][1]), np.ceil(u["x"][3]))
    assert b[2] == min(np.floor(u["y"][0]), np.floor(u["y"][1]))
    assert b[3] == max(np.ceil(u["y"][2]), np.ceil(u["y"][3]))


def frames():
    return synth.sequence(W, H, 3, seed=2024)


def oracle_frames():
    ex = RefExtractor(1000)
    out = []
    for f in frames():
        k, d = ex(f)
        out.append((ref_undistort(k), d))
    return out


def backproject(k, rng):
    z = rng.uniform(2.0, 6.0, len(k)).astype(np.float32)
    x = (k["x"] - K[2]) / K[0] * z
    y = (k["y"] - K[3]) / K[1] * z
    return np.ascontiguousarray(np.stack([x, y, z], 1).astype(np.float32))


POSE = np.array([[1, 0, 0.002, -0.006], [0, 1, 0, -0.003], [-0.002, 0, 1, 0.0]], np.float32).reshape(-1).copy()


@pytest.mark.gpu
def test_settings_camera_host_path_matches_oracle():
    """orbx_extract -> orbx_undistort_keypoints -> SearchForInitialization and
    the motion-model search on ComputeImageBounds' grid, host-pointer forms."""
    ref = oracle_frames()
    b = ref_bounds()
    ctx = ox.Context(nfeatures=1000, max_w=W, max_h=H, slots=1)
    L, R = ox.lib(), load()
    try:
        gpu = []
        for f, (rk, rd) in zip(frames(), ref):
            k, d = ctx(f)
            u = np.zeros_like(k)
            assert L.orbx_undistort_keypoints(ctx.handle, len(k), ox._ptr(k), ox._ptr(K), ox._ptr(DIST),
                                              ox._ptr(u)) == 0
            assert np.array_equal(u.view(np.uint8), rk.view(np.uint8)) and np.array_equal(d, rd)
            gpu.append((u, d))
        (k1, d1), (k2, d2), (k3, d3) = ref
        F1, F2 = view(k1, d1, b), view(k2, d2, b)
        prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
        pr, pg = prev.copy(), prev.copy()
        mr, mg = np.zeros(len(k1), np.int32), np.zeros(len(k1), np.int32)
        nr, ng = ctypes.c_int(), ctypes.c_int()
        assert R.orbx_ref_search_for_initialization(ctypes.byref(F1), ctypes.byref(F2), ptr(pr), ptr(mr), 100, 0.9, 1,
                                                    ctypes.byref(nr)) == 0
        assert L.orbx_search_for_initialization(ctx.handle, ctypes.byref(F1), ctypes.byref(F2), ox._ptr(pg),
                                                ox._ptr(mg), 100, 0.9, 1, ctypes.byref(ng)) == 0
        assert ng.value == nr.value > 0 and np.array_equal(mg, mr) and np.array_equal(pg, pr)
        # motion model: last frame 2, current frame 3
        C, Lv = view(k3, d3, b), F2
        rng = np.random.default_rng(5)
        xyz = backproject(k2, rng)
        valid = (rng.random(len(k2)) < 0.85).astype(np.uint8)
        assigned = np.zeros(len(k3), np.uint8)
        cam = K.copy()
        for th, ori in ((15.0, 1), (7.0, 0)):
            mr, mg = np.zeros(len(k3), np.int32), np.zeros(len(k3), np.int32)
            assert R.orbx_ref_search_by_projection_motion(ctypes.byref(C), ctypes.byref(Lv), ptr(xyz), ptr(valid),
                                                          ptr(assigned), ptr(POSE), ptr(cam), th, ori, ptr(mr),
                                                          ctypes.byref(nr)) == 0
            assert L.orbx_search_by_projection_motion(ctx.handle, ctypes.byref(C), ctypes.byref(Lv), ox._ptr(xyz),
                                                      ox._ptr(valid), ox._ptr(assigned), ox._ptr(POSE), ox._ptr(cam),
                                                      th, ori, ox._ptr(mg), ctypes.byref(ng)) == 0
            assert ng.value == nr.value > 0 and np.array_equal(mg, mr)
    finally:
        ctx.close()


@pytest.mark.gpu
def test_settings_camera_device_resident_matches_oracle():
    """The frames kept in slots: extraction, orbx_dev_undistort in place,
    orbx_dev_set_image_bounds with ComputeImageBounds' result, then the
    device SearchForInitialization of each slot against its predecessor."""
    ref = oracle_frames()
    b = ref_bounds()
    fr = frames()
    ctx = ox.Context(nfeatures=1000, max_w=W, max_h=H, slots=3)
    R = load()
    try:
        ctx.upload(fr)
        ctx.extract(0, 3)
        assert ox.lib().orbx_dev_undistort(ctx.handle, 0, 3, ox._ptr(K), ox._ptr(DIST)) == 0
        ctx.set_image_bounds(b)
        ctx.match_prev(0, 3, 3, window=100, nnratio=0.9, check_ori=True)
        ctx.sync()
        for s in range(3):
            gk, gd = ctx.features(s)
            rk, rd = ref[s]
            assert np.array_equal(gk.view(np.uint8), rk.view(np.uint8)) and np.array_equal(gd, rd)
        for s in (1, 2):
            (k1, d1), (k2, d2) = ref[s - 1], ref[s]
            F1, F2 = view(k1, d1, b), view(k2, d2, b)
            pr = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
            mr = np.zeros(len(k1), np.int32)
            nr = ctypes.c_int()
            assert R.orbx_ref_search_for_initialization(ctypes.byref(F1), ctypes.byref(F2), ptr(pr), ptr(mr), 100,
                                                        0.9, 1, ctypes.byref(nr)) == 0
            gm, gn = ctx.matches(s)
            assert gn == nr.value > 0 and np.array_equal(gm[:len(k1)], mr)
    finally:
        ctx.close()
