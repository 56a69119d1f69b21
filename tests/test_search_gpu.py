"""GPU parity of the ORBmatcher searches (host-pointer C-ABI entry points)
against the CPU restatement, on features of a synthetic sequence.

Covers SearchForInitialization (src/ORBmatcher.cc:598-713), WindowSearch
(:409-516), the three SearchByProjection variants (:49-125, :519-594,
:1507-1620) and brute-force Hamming matching (C3; rule of :640-654).
Results (match vectors and counts) must be identical.
"""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
from orb_slam_amd import synth
from oracle_lib import RefExtractor, load, ptr

pytestmark = pytest.mark.gpu

W, H = 640, 480
CAM = np.array([500.0, 500.0, 320.0, 240.0], np.float32)


@pytest.fixture(scope="module")
def frames_feats():
    frames = synth.sequence(W, H, 3, seed=77)
    ex = RefExtractor(1000)
    feats = [ex(f) for f in frames]
    return feats


@pytest.fixture(scope="module")
def ctx():
    c = ox.Context(nfeatures=1000, max_w=W, max_h=H, slots=1)
    yield c
    c.close()


def views(k1, d1, k2, d2):
    return ox.frame_view(k1, d1, W, H), ox.frame_view(k2, d2, W, H)


def backproject(k, rng):
    """World points for keypoints seen from the identity pose."""
    z = rng.uniform(2.0, 6.0, len(k)).astype(np.float32)
    x = (k["x"] - CAM[2]) / CAM[0] * z
    y = (k["y"] - CAM[3]) / CAM[1] * z
    return np.ascontiguousarray(np.stack([x, y, z], 1).astype(np.float32))


def pose(tx=-0.008, ty=-0.004, yaw=0.002):
    c, s = np.cos(yaw), np.sin(yaw)
    return np.array([[c, 0, s, tx], [0, 1, 0, ty], [-s, 0, c, 0.0]], np.float32).reshape(-1).copy()


@pytest.mark.parametrize("check_ori,window", [(True, 100), (False, 60)])
def test_search_for_initialization(ctx, frames_feats, check_ori, window):
    (k1, d1), (k2, d2) = frames_feats[0], frames_feats[1]
    F1, F2 = views(k1, d1, k2, d2)
    L = load()
    prev0 = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    pr, pg = prev0.copy(), prev0.copy()
    mr, mg = np.zeros(len(k1), np.int32), np.zeros(len(k1), np.int32)
    nr, ng = ctypes.c_int(), ctypes.c_int()
    assert L.orbx_ref_search_for_initialization(ctypes.byref(F1), ctypes.byref(F2), ptr(pr), ptr(mr), window, 0.9,
                                                int(check_ori), ctypes.byref(nr)) == 0
    assert ox.lib().orbx_search_for_initialization(ctx.handle, ctypes.byref(F1), ctypes.byref(F2), ox._ptr(pg),
                                                   ox._ptr(mg), window, 0.9, int(check_ori), ctypes.byref(ng)) == 0
    assert ng.value == nr.value and nr.value > 0
    assert np.array_equal(mg, mr)
    assert np.array_equal(pg, pr)


def _sfi_both(ctx, k1, d1, k2, d2, prev0, window, ratio, ori):
    F1, F2 = views(k1, d1, k2, d2)
    L = load()
    pr, pg = prev0.copy(), prev0.copy()
    mr, mg = np.zeros(len(k1), np.int32), np.zeros(len(k1), np.int32)
    nr, ng = ctypes.c_int(), ctypes.c_int()
    assert L.orbx_ref_search_for_initialization(ctypes.byref(F1), ctypes.byref(F2), ptr(pr), ptr(mr), window, ratio,
                                                int(ori), ctypes.byref(nr)) == 0
    assert ox.lib().orbx_search_for_initialization(ctx.handle, ctypes.byref(F1), ctypes.byref(F2), ox._ptr(pg),
                                                   ox._ptr(mg), window, ratio, int(ori), ctypes.byref(ng)) == 0
    assert ng.value == nr.value
    assert np.array_equal(mg, mr)
    assert np.array_equal(pg, pr)
    return nr.value


# the single-pair path (k_sfi_lists + k_search_init_one): lists longer than a
# wave (window 400: unsorted, reduction replay), short windows, ratios, moved
# search centres, and pairs without queries or without candidates
@pytest.mark.parametrize("pair,window,ratio,ori,jitter", [((0, 2), 400, 0.9, True, 0), ((1, 2), 20, 0.6, False, 0),
                                                          ((0, 1), 100, 1.0, True, 15), ((2, 0), 250, 0.8, True, 40),
                                                          ((1, 0), 0, 0.9, False, 0)])
def test_search_for_initialization_cases(ctx, frames_feats, pair, window, ratio, ori, jitter):
    (k1, d1), (k2, d2) = frames_feats[pair[0]], frames_feats[pair[1]]
    rng = np.random.default_rng(window + jitter)
    prev0 = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    prev0 += rng.uniform(-jitter, jitter, prev0.shape).astype(np.float32)
    n = _sfi_both(ctx, k1, d1, k2, d2, prev0, window, ratio, ori)
    if window >= 100:
        assert n > 0


@pytest.mark.parametrize("which", ["no_queries", "no_candidates"])
def test_search_for_initialization_empty(ctx, frames_feats, which):
    (k1, d1), (k2, d2) = frames_feats[0], frames_feats[1]
    k1, k2 = k1.copy(), k2.copy()
    (k1 if which == "no_queries" else k2)["octave"] = np.maximum((k1 if which == "no_queries" else k2)["octave"], 1)
    prev0 = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    assert _sfi_both(ctx, k1, d1, k2, d2, prev0, 100, 0.9, True) == 0


# the two-phase searches (k_area_lists + k_area_replay): short sorted lists,
# lists of 65..128 candidates in index order, and longer ones that the replay
# evaluates in full (windows of 100 .. 400 pixels)
@pytest.mark.parametrize("window,minl,maxl,ratio,ori", [(100, 0, -1, 0.9, True), (200, 1, 5, 0.7, False),
                                                         (30, 0, 2, 1.0, True), (400, 0, -1, 0.8, True),
                                                         (60, 0, -1, 0.9, False)])
def test_window_search(ctx, frames_feats, window, minl, maxl, ratio, ori):
    (k1, d1), (k2, d2) = frames_feats[0], frames_feats[1]
    F1, F2 = views(k1, d1, k2, d2)
    rng = np.random.default_rng(window)
    mp = (rng.random(len(k1)) < 0.7).astype(np.uint8)
    mr, mg = np.zeros(len(k2), np.int32), np.zeros(len(k2), np.int32)
    nr, ng = ctypes.c_int(), ctypes.c_int()
    assert load().orbx_ref_window_search(ctypes.byref(F1), ctypes.byref(F2), ptr(mp), window, minl, maxl, ratio,
                                         int(ori), ptr(mr), ctypes.byref(nr)) == 0
    assert ox.lib().orbx_window_search(ctx.handle, ctypes.byref(F1), ctypes.byref(F2), ox._ptr(mp), window, minl,
                                       maxl, ratio, int(ori), ox._ptr(mg), ctypes.byref(ng)) == 0
    assert ng.value == nr.value and nr.value > 0
    assert np.array_equal(mg, mr)


@pytest.mark.parametrize("window", [15, 50, 150, 300])
def test_search_by_projection_pair(ctx, frames_feats, window):
    (k1, d1), (k2, d2) = frames_feats[0], frames_feats[1]
    F1, F2 = views(k1, d1, k2, d2)
    rng = np.random.default_rng(window)
    xyz = backproject(k1, rng)
    valid = (rng.random(len(k1)) < 0.8).astype(np.uint8)
    assigned = (rng.random(len(k2)) < 0.1).astype(np.uint8)
    T = pose()
    mr, mg = np.zeros(len(k2), np.int32), np.zeros(len(k2), np.int32)
    nr, ng = ctypes.c_int(), ctypes.c_int()
    assert load().orbx_ref_search_by_projection_pair(ctypes.byref(F1), ctypes.byref(F2), ptr(xyz), ptr(valid),
                                                     ptr(assigned), ptr(T), ptr(CAM), window, 0.9, ptr(mr),
                                                     ctypes.byref(nr)) == 0
    assert ox.lib().orbx_search_by_projection_pair(ctx.handle, ctypes.byref(F1), ctypes.byref(F2), ox._ptr(xyz),
                                                   ox._ptr(valid), ox._ptr(assigned), ox._ptr(T), ox._ptr(CAM),
                                                   window, 0.9, ox._ptr(mg), ctypes.byref(ng)) == 0
    assert ng.value == nr.value and nr.value > 0
    assert np.array_equal(mg, mr)


@pytest.mark.parametrize("th,ori", [(15.0, True), (7.0, False), (40.0, True), (120.0, False), (2.0, True)])
def test_search_by_projection_motion(ctx, frames_feats, th, ori):
    (kl, dl), (kc, dc) = frames_feats[1], frames_feats[2]
    C, Lv = views(kc, dc, kl, dl)
    rng = np.random.default_rng(int(th))
    xyz = backproject(kl, rng)
    valid = (rng.random(len(kl)) < 0.85).astype(np.uint8)
    assigned = np.zeros(len(kc), np.uint8)
    T = pose()
    mr, mg = np.zeros(len(kc), np.int32), np.zeros(len(kc), np.int32)
    nr, ng = ctypes.c_int(), ctypes.c_int()
    assert load().orbx_ref_search_by_projection_motion(ctypes.byref(C), ctypes.byref(Lv), ptr(xyz), ptr(valid),
                                                       ptr(assigned), ptr(T), ptr(CAM), th, int(ori), ptr(mr),
                                                       ctypes.byref(nr)) == 0
    assert ox.lib().orbx_search_by_projection_motion(ctx.handle, ctypes.byref(C), ctypes.byref(Lv), ox._ptr(xyz),
                                                     ox._ptr(valid), ox._ptr(assigned), ox._ptr(T), ox._ptr(CAM),
                                                     th, int(ori), ox._ptr(mg), ctypes.byref(ng)) == 0
    assert ng.value == nr.value and nr.value > 0
    assert np.array_equal(mg, mr)


@pytest.mark.parametrize("th", [1.0, 5.0, 12.0, 30.0])
def test_search_by_projection_local(ctx, frames_feats, th):
    (km, dm), (kf, df) = frames_feats[0], frames_feats[1]
    F = ox.frame_view(kf, df, W, H)
    rng = np.random.default_rng(int(th * 10))
    n = len(km)
    in_view = (rng.random(n) < 0.9).astype(np.uint8)
    proj = np.ascontiguousarray(np.stack([km["x"] + 2.0, km["y"] + 1.0], 1).astype(np.float32))
    pred = np.ascontiguousarray(km["octave"].astype(np.int32))
    vcos = rng.uniform(0.99, 1.0, n).astype(np.float32)
    mpd = np.ascontiguousarray(dm)
    assigned = (rng.random(len(kf)) < 0.05).astype(np.uint8)
    mr, mg = np.zeros(len(kf), np.int32), np.zeros(len(kf), np.int32)
    nr, ng = ctypes.c_int(), ctypes.c_int()
    assert load().orbx_ref_search_by_projection_local(ctypes.byref(F), n, ptr(in_view), ptr(proj), ptr(pred),
                                                      ptr(vcos), ptr(mpd), ptr(assigned), th, 0.8, ptr(mr),
                                                      ctypes.byref(nr)) == 0
    assert ox.lib().orbx_search_by_projection_local(ctx.handle, ctypes.byref(F), n, ox._ptr(in_view), ox._ptr(proj),
                                                    ox._ptr(pred), ox._ptr(vcos), ox._ptr(mpd), ox._ptr(assigned),
                                                    th, 0.8, ox._ptr(mg), ctypes.byref(ng)) == 0
    assert ng.value == nr.value and nr.value > 0
    assert np.array_equal(mg, mr)


@pytest.mark.parametrize("na,nb", [(1000, 1000), (2000, 1999), (1, 300), (257, 0), (0, 100), (65, 63), (3000, 4500),
                                   (4097, 2)])
def test_hamming_bf_and_match(ctx, na, nb):
    rng = np.random.default_rng(na + nb)
    dA = rng.integers(0, 256, (na, 32), dtype=np.uint8)
    dB = rng.integers(0, 256, (nb, 32), dtype=np.uint8)
    # plant near-duplicates and exact ties
    k = min(na, nb) // 2
    if k:
        dB[:k] = dA[:k] ^ (rng.random((k, 32)) < 0.03).astype(np.uint8)
        dB[k // 2:k] = dB[:k - k // 2] if nb > 1 else dB[k // 2:k]
    dA, dB = np.ascontiguousarray(dA), np.ascontiguousarray(dB)
    ri, r1, r2 = (np.zeros(na, np.int32) for _ in range(3))
    gi, g1, g2 = (np.zeros(na, np.int32) for _ in range(3))
    assert load().orbx_ref_hamming_bf(ptr(dA), na, ptr(dB), nb, ptr(ri), ptr(r1), ptr(r2)) == 0
    assert ox.lib().orbx_hamming_bf(ctx.handle, ox._ptr(dA), na, ox._ptr(dB), nb, ox._ptr(gi), ox._ptr(g1),
                                    ox._ptr(g2)) == 0
    assert np.array_equal(gi, ri) and np.array_equal(g1, r1) and np.array_equal(g2, r2)
    m = np.zeros(na, np.int32)
    nm = ctypes.c_int()
    assert ox.lib().orbx_match_bf(ctx.handle, ox._ptr(dA), na, ox._ptr(dB), nb, 50, 0.9, ox._ptr(m),
                                  ctypes.byref(nm)) == 0
    ok = (r1 <= 50) & (r1.astype(np.float32) < r2.astype(np.float32) * np.float32(0.9))
    assert np.array_equal(m, np.where(ok, ri, -1))
    assert nm.value == int(ok.sum())
