"""Frame::UndistortKeyPoints / ComputeImageBounds (src/Frame.cc:288-348):
the CPU restatement (oracle/ref_frame.cpp) inverts the Brown-Conrady model
(checked against a numpy forward distortion), and the GPU path matches it
bit for bit (host-pointer and device-resident forms)."""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
from oracle_lib import load, ptr

K = np.array([517.3, 516.5, 318.6, 255.3], np.float32)        # TUM fr1-like intrinsics
DIST = np.array([0.2624, -0.9531, -0.0054, 0.0026, 1.1633], np.float32)


def keys(n=1000, seed=0):
    rng = np.random.default_rng(seed)
    k = np.zeros(n, ox.KEYPOINT)
    k["x"] = rng.uniform(0, 640, n)
    k["y"] = rng.uniform(0, 480, n)
    k["angle"] = rng.uniform(0, 360, n)
    k["octave"] = rng.integers(0, 8, n)
    k["class_id"] = -1
    return k


def ref_undistort(k, dist):
    L = load()
    L.orbx_ref_undistort_keypoints.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4
    out = np.zeros_like(k)
    assert L.orbx_ref_undistort_keypoints(len(k), ptr(k), ptr(K), ptr(dist), ptr(out)) == 0
    return out


def distort(x, y, d):
    """Forward Brown-Conrady on normalised coordinates."""
    k1, k2, p1, p2, k3 = [float(v) for v in d]
    r2 = x * x + y * y
    rad = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 ** 3
    return (x * rad + 2 * p1 * x * y + p2 * (r2 + 2 * x * x), y * rad + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y)


def test_undistort_inverts_the_distortion_model():
    d = np.array([0.05, -0.02, 0.001, -0.0005, 0.0], np.float32)
    rng = np.random.default_rng(1)
    xu, yu = rng.uniform(-0.5, 0.5, 200), rng.uniform(-0.4, 0.4, 200)
    xd, yd = distort(xu, yu, d)
    k = np.zeros(200, ox.KEYPOINT)
    k["x"], k["y"] = xd * K[0] + K[2], yd * K[1] + K[3]
    out = ref_undistort(k, d)
    assert np.abs(out["x"] - (xu * K[0] + K[2])).max() < 0.05
    assert np.abs(out["y"] - (yu * K[1] + K[3])).max() < 0.05
    assert np.array_equal(out["angle"], k["angle"]) and np.array_equal(out["octave"], k["octave"])


def test_zero_k1_copies_and_bounds_are_the_image():
    k = keys(50)
    d = np.array([0.0, 0.3, 0.1, 0.1, 0.0], np.float32)
    assert np.array_equal(ref_undistort(k, d), k)
    L = load()
    L.orbx_ref_compute_image_bounds.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 3
    b = np.zeros(4, np.float32)
    assert L.orbx_ref_compute_image_bounds(640, 480, ptr(K), ptr(d), ptr(b)) == 0
    assert list(b) == [0, 640, 0, 480]
    g = np.zeros(4, np.float32)
    assert ox.lib().orbx_compute_image_bounds(640, 480, ox._ptr(K), ox._ptr(d), ox._ptr(g)) == 0
    assert list(g) == [0, 640, 0, 480]


def test_image_bounds_host_matches_oracle():
    L = load()
    L.orbx_ref_compute_image_bounds.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 3
    b, g = np.zeros(4, np.float32), np.zeros(4, np.float32)
    assert L.orbx_ref_compute_image_bounds(640, 480, ptr(K), ptr(DIST), ptr(b)) == 0
    assert ox.lib().orbx_compute_image_bounds(640, 480, ox._ptr(K), ox._ptr(DIST), ox._ptr(g)) == 0
    assert np.array_equal(b, g) and list(b) != [0, 640, 0, 480]


@pytest.mark.gpu
def test_gpu_undistort_matches_oracle():
    ctx = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
    try:
        for seed, d in [(0, DIST), (1, np.array([-0.3, 0.1, 0.0, 0.0, 0.0], np.float32))]:
            k = keys(3000, seed)
            r = ref_undistort(k, d)
            g = np.zeros_like(k)
            assert ox.lib().orbx_undistort_keypoints(ctx.handle, len(k), ox._ptr(k), ox._ptr(K), ox._ptr(d),
                                                     ox._ptr(g)) == 0
            assert np.array_equal(g, r)
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_dev_undistort_slots():
    from orb_slam_amd import synth
    w, h = 320, 240
    frames = synth.sequence(w, h, 3, seed=9)
    ctx = ox.Context(nfeatures=500, max_w=w, max_h=h, slots=3)
    try:
        ctx.upload(frames)
        ctx.extract(0, 3)
        ctx.sync()
        raw = [ctx.features(s)[0] for s in range(3)]
        assert ox.lib().orbx_dev_undistort(ctx.handle, 0, 3, ox._ptr(K), ox._ptr(DIST)) == 0
        ctx.sync()
        for s in range(3):
            g = ctx.features(s)[0]
            assert len(g) == len(raw[s]) > 0
            assert np.array_equal(g, ref_undistort(raw[s], DIST))
    finally:
        ctx.close()
