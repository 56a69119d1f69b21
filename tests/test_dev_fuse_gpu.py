"""Fuse against keyframes resident in their extraction slots
(orbx_dev_fuse_candidates; LocalMapping::SearchInNeighbors' loop,
src/LocalMapping.cc:403-416, over ORBmatcher::Fuse, src/ORBmatcher.cc:
1016-1265) through the C ABI against the CPU restatement: best keypoint and
distance of every map point identical, for several keyframes in one call,
with and without explicit image bounds, both Fuse overloads."""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
import proj_data as pd
from orb_slam_amd import synth
from test_proj_oracle import ref_fuse

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def slots():
    c = ox.Context(nfeatures=1000, max_w=pd.W, max_h=pd.H, slots=3)
    frames = np.stack(synth.sequence(pd.W, pd.H, 2, seed=31))
    c.upload(frames, 0)
    c.upload(synth.texture_frame(pd.W, pd.H, seed=8), 2)
    c.extract(0, 3)
    c.sync()
    yield c, [c.features(s) for s in range(3)]
    c.close()


def dev_fuse(c, slots_, bounds, views, Ts, sim3, th):
    n = len(slots_)
    sl = np.ascontiguousarray(slots_ or [0], np.int32)
    cams = np.ascontiguousarray(np.tile(pd.CAM, n).astype(np.float32))
    Tall = np.ascontiguousarray(np.concatenate([T.reshape(-1) for T in Ts] or [np.zeros(16)]).astype(np.float32))
    mpp = (ctypes.c_void_p * max(n, 1))(*[ctypes.addressof(v) for v in views])
    bis = [np.zeros(v.n, np.int32) for v in views]
    bds = [np.zeros(v.n, np.int32) for v in views]
    bip = (ctypes.c_void_p * max(n, 1))(*[b.ctypes.data for b in bis])
    bdp = (ctypes.c_void_p * max(n, 1))(*[b.ctypes.data for b in bds])
    b = None if bounds is None else np.ascontiguousarray(bounds, np.float32)
    r = ox.lib().orbx_dev_fuse_candidates(c.handle, n, ox._ptr(sl), ox._ptr(b) if b is not None else None,
                                          ox._ptr(cams), mpp, ox._ptr(Tall), sim3, th, bip, bdp)
    return r, bis, bds


@pytest.mark.parametrize("sim3,th,with_bounds", [(0, 3.0, False), (1, 5.0, False), (0, 7.5, True), (1, 3.0, True)])
def test_dev_fuse_matches_oracle(slots, sim3, th, with_bounds):
    c, feats = slots
    (k0, d0), (k1, d1), (k2, d2) = feats
    du = float(np.median(k1["x"])) - float(np.median(k0["x"]))   # rough shift; the oracle decides parity
    rng = np.random.default_rng(int(10 * th) + sim3)
    mps = pd.mappoints(k0, d0, pd.pose_T([0, 0, 0]), rng)
    mps[1]["pos"][:20, 2] *= -1
    mps[1]["max_dist"][20:40] *= 0.1
    other = pd.mappoints(k2, d2, pd.pose_T([0, 0, 0]), np.random.default_rng(5))
    _, _, _, _, sdu, sdv = pd.keyframes()
    T1 = pd.pose_T([sdu * pd.Z0 / pd.CAM[0], sdv * pd.Z0 / pd.CAM[1], 0.0])
    Ts = [T1, pd.pose_T([0, 0, 0]), T1 + 0, pd.pose_T([0.01, 0, 0.002])]
    if sim3:
        Ts = [T.copy() for T in Ts]
        for T in Ts:
            T[:3, :] *= np.float32(1.3)
    kf_slots = [1, 0, 2, 2]
    views = [mps[0], mps[0], mps[0], other[0]]
    sets = [mps, mps, mps, other]
    bounds = None
    if with_bounds:
        bounds = np.array([[2.0, pd.W - 3.0, 1.0, pd.H - 2.0]] * len(kf_slots), np.float32).reshape(-1)
    r, bis, bds = dev_fuse(c, kf_slots, bounds, views, Ts, sim3, th)
    assert r == 0, r
    for k, sl in enumerate(kf_slots):
        kk, kd = feats[sl]
        KF = ox.frame_view(kk, kd, pd.W, pd.H)
        if with_bounds:
            KF.min_x, KF.max_x, KF.min_y, KF.max_y = bounds[4 * k:4 * k + 4]
        rb = ref_fuse(KF, sets[k], Ts[k], sim3, th)
        assert np.array_equal(bis[k], rb[0]) and np.array_equal(bds[k], rb[1]), k
    assert (bds[1] <= 50).sum() > 100   # the points fused back into their own keyframe


def test_dev_fuse_errors(slots):
    c, feats = slots
    k0, d0 = feats[0]
    mps = pd.mappoints(k0, d0, pd.pose_T([0, 0, 0]), np.random.default_rng(1))
    T = pd.pose_T([0, 0, 0])
    assert dev_fuse(c, [], None, [], [], 0, 3.0)[0] == 0
    assert dev_fuse(c, [3], None, [mps[0]], [T], 0, 3.0)[0] == -1                    # no such slot
    assert dev_fuse(c, [0], [5.0, 5.0, 0.0, 10.0], [mps[0]], [T], 0, 3.0)[0] == -1   # empty bounds


@pytest.mark.parametrize("seed,th,scale,with_bounds", [(0, 10, 1.5, False), (1, 5, 1.0, True), (2, 20, 0.8, False)])
def test_dev_search_by_projection_kf_sim3_matches_oracle(slots, seed, th, scale, with_bounds):
    """SearchByProjection(pKF, Scw, ...) against the keyframe in slot 1, map
    points from slot 0's keypoints: matched vector and count as the oracle."""
    from test_proj_oracle import ref_proj_kf_sim3
    c, feats = slots
    (k0, d0), (k1, d1) = feats[0], feats[1]
    _, _, _, _, du, dv = pd.keyframes()
    rng = np.random.default_rng(seed)
    mps = pd.mappoints(k0, d0, pd.pose_T([0, 0, 0]), rng)
    S = pd.pose_T([du * pd.Z0 / pd.CAM[0], dv * pd.Z0 / pd.CAM[1], 0.0])
    S[:3, :] *= np.float32(scale)
    skip = (rng.random(len(k0)) < 0.1).astype(np.uint8)
    matched = np.full(len(k1), -1, np.int32)
    matched[rng.random(len(k1)) < 0.05] = 10 ** 6
    KF = ox.frame_view(k1, d1, pd.W, pd.H)
    b = None
    if with_bounds:
        b = np.array([1.0, pd.W - 2.0, 3.0, pd.H - 1.0], np.float32)
        KF.min_x, KF.max_x, KF.min_y, KF.max_y = b
    ro, rn = ref_proj_kf_sim3(KF, mps, skip, S, th, matched)
    go = np.full(c.nfeatures, -7, np.int32)
    go[:len(k1)] = matched
    gn = ctypes.c_int()
    assert ox.lib().orbx_dev_search_by_projection_kf_sim3(c.handle, 1, ox._ptr(b) if b is not None else None,
                                                          ox._ptr(pd.CAM), ctypes.byref(mps[0]), ox._ptr(skip),
                                                          ox._ptr(S), th, ox._ptr(go), c.nfeatures,
                                                          ctypes.byref(gn)) == 0
    assert gn.value == rn and rn > 50
    assert np.array_equal(go[:len(k1)], ro) and np.all(go[len(k1):] == -7)
    # capacity below the slot's keypoint count
    assert ox.lib().orbx_dev_search_by_projection_kf_sim3(c.handle, 1, None, ox._ptr(pd.CAM), ctypes.byref(mps[0]),
                                                          ox._ptr(skip), ox._ptr(S), th, ox._ptr(go), len(k1) - 1,
                                                          ctypes.byref(gn)) == -3


@pytest.mark.parametrize("seed,th,orb,ori,with_bounds", [(0, 10.0, 100, 1, False), (1, 5.0, 64, 0, True),
                                                          (2, 15.0, 50, 1, False)])
def test_dev_search_by_projection_frame_kf_matches_oracle(slots, seed, th, orb, ori, with_bounds):
    """Relocalisation's SearchByProjection(CurrentFrame, pKF, sAlreadyFound)
    with the frame in slot 1 and the keyframe in slot 0 (map points of the
    keyframe's keypoints): matches and count as the oracle."""
    from test_proj_oracle import ref_proj_frame_kf
    c, feats = slots
    (k0, d0), (k1, d1) = feats[0], feats[1]
    _, _, _, _, du, dv = pd.keyframes()
    rng = np.random.default_rng(seed)
    mps = pd.mappoints(k0, d0, pd.pose_T([0, 0, 0]), rng)
    T = pd.pose_T([du * pd.Z0 / pd.CAM[0], dv * pd.Z0 / pd.CAM[1], 0.0])
    valid = (rng.random(len(k0)) < 0.8).astype(np.uint8)
    assigned = (rng.random(len(k1)) < 0.1).astype(np.uint8)
    F, KF = ox.frame_view(k1, d1, pd.W, pd.H), ox.frame_view(k0, d0, pd.W, pd.H)
    b = None
    if with_bounds:
        b = np.array([2.0, pd.W - 1.0, 0.0, pd.H - 3.0], np.float32)
        F.min_x, F.max_x, F.min_y, F.max_y = b
    ro, rn = ref_proj_frame_kf(F, KF, mps, valid, assigned, T, th, orb, ori)
    go = np.full(c.nfeatures, -7, np.int32)
    gn = ctypes.c_int()
    assert ox.lib().orbx_dev_search_by_projection_frame_kf(c.handle, 1, ox._ptr(b) if b is not None else None, 0,
                                                           ox._ptr(pd.CAM), ctypes.byref(mps[0]), ox._ptr(valid),
                                                           ox._ptr(assigned), ox._ptr(T), th, orb, ori, ox._ptr(go),
                                                           c.nfeatures, ctypes.byref(gn)) == 0
    assert gn.value == rn and rn > 50
    assert np.array_equal(go[:len(k1)], ro) and np.all(go[len(k1):] == -7)
    # the keyframe's map points must be one per keyframe keypoint
    short = pd.mappoints(k0[:10], d0[:10], pd.pose_T([0, 0, 0]), rng)
    assert ox.lib().orbx_dev_search_by_projection_frame_kf(c.handle, 1, None, 0, ox._ptr(pd.CAM),
                                                           ctypes.byref(short[0]), ox._ptr(valid), ox._ptr(assigned),
                                                           ox._ptr(T), th, orb, ori, ox._ptr(go), c.nfeatures,
                                                           ctypes.byref(gn)) == -1


@pytest.mark.parametrize("seed,th,prior,with_bounds", [(0, 7.5, 0.1, False), (1, 4.0, 0.0, True), (2, 10.0, 0.4, False)])
def test_dev_search_by_sim3_matches_oracle(slots, seed, th, prior, with_bounds):
    """LoopClosing's SearchBySim3 with KF1 in slot 0 and KF2 in slot 1:
    the agreed matches and their count as the oracle."""
    from test_proj_oracle import ref_sim3
    c, feats = slots
    (k1, d1), (k2, d2) = feats[0], feats[1]
    _, _, _, _, du, dv = pd.keyframes()
    rng = np.random.default_rng(seed)
    t2 = np.array([du * pd.Z0 / pd.CAM[0], dv * pd.Z0 / pd.CAM[1], 0.0], np.float32)
    T1, T2 = pd.pose_T([0, 0, 0]), pd.pose_T(t2)
    m1 = pd.mappoints(k1, d1, T1, rng)
    m2 = pd.mappoints(k2, d2, T2, rng)
    v1 = (rng.random(len(k1)) < 0.85).astype(np.uint8)
    v2 = (rng.random(len(k2)) < 0.85).astype(np.uint8)
    pr = np.full(len(k1), -2, np.int32)
    sel = rng.random(len(k1)) < prior
    pr[sel] = rng.integers(-1, len(k2), sel.sum())
    R12 = np.eye(3, dtype=np.float32)
    t12 = (-t2).astype(np.float32)
    K1, K2 = ox.frame_view(k1, d1, pd.W, pd.H), ox.frame_view(k2, d2, pd.W, pd.H)
    b1 = b2 = None
    if with_bounds:
        b1 = np.array([1.0, pd.W - 2.0, 2.0, pd.H - 1.0], np.float32)
        b2 = np.array([0.0, pd.W - 3.0, 1.0, pd.H - 2.0], np.float32)
        K1.min_x, K1.max_x, K1.min_y, K1.max_y = b1
        K2.min_x, K2.max_x, K2.min_y, K2.max_y = b2
    rn, rc = ref_sim3(K1, K2, m1, v1, m2, v2, T1, T2, np.float32(1.0), R12, t12, pr, th)
    gn = np.full(c.nfeatures, -7, np.int32)
    gc = ctypes.c_int()
    bp = lambda b: ox._ptr(b) if b is not None else None
    assert ox.lib().orbx_dev_search_by_sim3(c.handle, 0, bp(b1), 1, bp(b2), ox._ptr(pd.CAM), ctypes.byref(m1[0]),
                                            ox._ptr(v1), ctypes.byref(m2[0]), ox._ptr(v2), ox._ptr(T1), ox._ptr(T2),
                                            1.0, ox._ptr(R12), ox._ptr(t12), th, ox._ptr(pr), ox._ptr(gn), c.nfeatures,
                                            ctypes.byref(gc)) == 0
    assert gc.value == rc and rc > 50
    assert np.array_equal(gn[:len(k1)], rn) and np.all(gn[len(k1):] == -7)
