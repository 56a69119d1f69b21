"""GPU keyframe projection searches through the C ABI against the CPU
restatement (oracle/ref_proj.cpp): Fuse's per-point candidates (both
overloads, src/ORBmatcher.cc:1016-1265), SearchBySim3 (:1267-1505) and
ComputeDistinctiveDescriptors (src/MapPoint.cc:185-250).  Results must be
identical."""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
import proj_data as pd
from test_proj_oracle import ref_distinctive, ref_fuse, ref_sim3, sim3_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
    yield c
    c.close()


def gpu_fuse(ctx, KF, mps, T, sim3, th):
    n = mps[0].n
    bi, bd = np.zeros(n, np.int32), np.zeros(n, np.int32)
    assert ox.lib().orbx_fuse_candidates(ctx.handle, ctypes.byref(KF), ox._ptr(pd.CAM), ctypes.byref(mps[0]),
                                         ox._ptr(T), sim3, th, ox._ptr(bi), ox._ptr(bd)) == 0
    return bi, bd


@pytest.mark.parametrize("sim3,th,seed", [(0, 3.0, 0), (0, 5.0, 1), (1, 3.0, 2), (1, 10.0, 3), (0, 2.0, 4), (1, 7.5, 5),
                                          (0, 12.0, 6), (1, 4.0, 7)])
def test_fuse_candidates_match_oracle(ctx, sim3, th, seed):
    k1, d1, k2, d2, du, dv = pd.keyframes()
    rng = np.random.default_rng(seed)
    T2 = pd.pose_T([du * pd.Z0 / pd.CAM[0], dv * pd.Z0 / pd.CAM[1], 0.0])
    mps = pd.mappoints(k1, d1, pd.pose_T([0, 0, 0]), rng)
    # points behind the camera and far outside the distance range
    mps[1]["pos"][:20, 2] *= -1
    mps[1]["max_dist"][20:40] *= 0.1
    T = T2.copy()
    if sim3:
        T[:3, :] *= np.float32(1.7)
    KF = pd.view(k2, d2)
    rb = ref_fuse(KF, mps, T, sim3, th)
    gb = gpu_fuse(ctx, KF, mps, T, sim3, th)
    assert (rb[1] <= 50).sum() > 100
    assert np.array_equal(gb[0], rb[0]) and np.array_equal(gb[1], rb[1])


@pytest.mark.parametrize("seed,th,prior", [(0, 7.5, 0.1), (1, 4.0, 0.0), (2, 10.0, 0.4), (3, 6.0, 0.2), (4, 9.0, 0.0),
                                           (5, 3.0, 0.3)])
def test_search_by_sim3_matches_oracle(ctx, seed, th, prior):
    c = sim3_case(seed, prior)
    K1, K2, m1, v1, m2, v2, T1, T2, s12, R12, t12, pr = c[:12]
    rn, rc = ref_sim3(K1, K2, m1, v1, m2, v2, T1, T2, s12, R12, t12, pr, th)
    gn = np.zeros(K1.n, np.int32)
    gc = ctypes.c_int()
    assert ox.lib().orbx_search_by_sim3(ctx.handle, ctypes.byref(K1), ctypes.byref(K2), ox._ptr(pd.CAM),
                                        ctypes.byref(m1[0]), ox._ptr(v1), ctypes.byref(m2[0]), ox._ptr(v2),
                                        ox._ptr(T1), ox._ptr(T2), float(s12), ox._ptr(R12), ox._ptr(t12), th,
                                        ox._ptr(pr), ox._ptr(gn), ctypes.byref(gc)) == 0
    assert gc.value == rc and rc > 50
    assert np.array_equal(gn, rn)


@pytest.mark.parametrize("seed", [0, 1, 2, 3, 4])
def test_distinctive_descriptors_match_oracle(ctx, seed):
    p, d = pd.distinctive_sets(n_mp=600, seed=seed)
    rb = ref_distinctive(p, d)
    gb = np.zeros(len(p) - 1, np.int32)
    assert ox.lib().orbx_distinctive_descriptors(ctx.handle, len(p) - 1, ox._ptr(p), ox._ptr(d), ox._ptr(gb)) == 0
    assert np.array_equal(gb, rb)


@pytest.mark.parametrize("seed,th,scale", [(0, 10, 1.5), (1, 5, 1.0), (2, 20, 0.8), (3, 8, 1.2), (4, 12, 0.9),
                                           (5, 15, 2.0)])
def test_search_by_projection_kf_sim3_matches_oracle(ctx, seed, th, scale):
    from test_proj_oracle import ref_proj_kf_sim3, seq_case
    k1, d1, k2, d2, T2, mps, rng = seq_case(seed)
    S = T2.copy()
    S[:3, :] *= np.float32(scale)
    skip = (rng.random(len(k1)) < 0.1).astype(np.uint8)
    matched = np.full(len(k2), -1, np.int32)
    matched[rng.random(len(k2)) < 0.05] = 10 ** 6
    KF = pd.view(k2, d2)
    ro, rn = ref_proj_kf_sim3(KF, mps, skip, S, th, matched)
    go = matched.copy()
    gn = ctypes.c_int()
    assert ox.lib().orbx_search_by_projection_kf_sim3(ctx.handle, ctypes.byref(KF), ox._ptr(pd.CAM),
                                                      ctypes.byref(mps[0]), ox._ptr(skip), ox._ptr(S), th,
                                                      ox._ptr(go), ctypes.byref(gn)) == 0
    assert gn.value == rn and rn > 100
    assert np.array_equal(go, ro)


@pytest.mark.parametrize("seed,th,orb,ori", [(0, 10.0, 100, 1), (1, 5.0, 64, 0), (2, 15.0, 50, 1), (3, 7.0, 80, 0),
                                              (4, 20.0, 100, 1), (5, 9.0, 40, 1)])
def test_search_by_projection_frame_kf_matches_oracle(ctx, seed, th, orb, ori):
    from test_proj_oracle import ref_proj_frame_kf, seq_case
    k1, d1, k2, d2, T2, mps, rng = seq_case(seed)
    valid = (rng.random(len(k1)) < 0.8).astype(np.uint8)
    assigned = (rng.random(len(k2)) < 0.1).astype(np.uint8)
    F, KF = pd.view(k2, d2), pd.view(k1, d1)
    ro, rn = ref_proj_frame_kf(F, KF, mps, valid, assigned, T2, th, orb, ori)
    go = np.zeros(len(k2), np.int32)
    gn = ctypes.c_int()
    assert ox.lib().orbx_search_by_projection_frame_kf(ctx.handle, ctypes.byref(F), ctypes.byref(KF),
                                                       ox._ptr(pd.CAM), ctypes.byref(mps[0]), ox._ptr(valid),
                                                       ox._ptr(assigned), ox._ptr(T2), th, orb, ori, ox._ptr(go),
                                                       ctypes.byref(gn)) == 0
    assert gn.value == rn and rn > 100
    assert np.array_equal(go, ro)
