"""CPU checks of the keyframe projection restatements (oracle/ref_proj.cpp):
Fuse's candidates, SearchBySim3 and ComputeDistinctiveDescriptors."""
import ctypes

import numpy as np

from oracle_lib import load, ptr
import proj_data as pd


def ref_fuse(KF, mps, T, sim3, th=3.0):
    n = mps[0].n
    bi, bd = np.zeros(n, np.int32), np.zeros(n, np.int32)
    L = load()
    L.orbx_ref_fuse_candidates.argtypes = [ctypes.c_void_p] * 8 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_float,
                                                                   ctypes.c_void_p, ctypes.c_void_p]
    a = mps[1]
    assert L.orbx_ref_fuse_candidates(ctypes.byref(KF), ptr(pd.CAM), n, ptr(a["pos"]), ptr(a["normal"]),
                                      ptr(a["min_dist"]), ptr(a["max_dist"]), ptr(a["desc"]), ptr(T), sim3, th,
                                      ptr(bi), ptr(bd)) == 0
    return bi, bd


def ref_sim3(K1, K2, m1, v1, m2, v2, T1, T2, s12, R12, t12, prior, th=7.5):
    L = load()
    L.orbx_ref_search_by_sim3.argtypes = ([ctypes.c_void_p] * 15 + [ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
                                                                   ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
                                                                   ctypes.c_void_p])
    new = np.zeros(K1.n, np.int32)
    n = ctypes.c_int()
    a, b = m1[1], m2[1]
    assert L.orbx_ref_search_by_sim3(ctypes.byref(K1), ctypes.byref(K2), ptr(pd.CAM), ptr(a["pos"]),
                                     ptr(a["min_dist"]), ptr(a["max_dist"]), ptr(a["desc"]), ptr(v1), ptr(b["pos"]),
                                     ptr(b["min_dist"]), ptr(b["max_dist"]), ptr(b["desc"]), ptr(v2), ptr(T1),
                                     ptr(T2), s12, ptr(R12), ptr(t12), th, ptr(prior), ptr(new),
                                     ctypes.byref(n)) == 0
    return new, n.value


def ref_distinctive(p, d):
    best = np.zeros(len(p) - 1, np.int32)
    L = load()
    L.orbx_ref_distinctive_descriptors.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    assert L.orbx_ref_distinctive_descriptors(len(p) - 1, ptr(p), ptr(d), ptr(best)) == 0
    return best


def sim3_case(seed=0, prior_frac=0.1):
    k1, d1, k2, d2, du, dv = pd.keyframes()
    rng = np.random.default_rng(seed)
    t2 = np.array([du * pd.Z0 / pd.CAM[0], dv * pd.Z0 / pd.CAM[1], 0.0], np.float32)
    T1, T2 = pd.pose_T([0, 0, 0]), pd.pose_T(t2)
    m1 = pd.mappoints(k1, d1, T1, rng)
    m2 = pd.mappoints(k2, d2, T2, rng)
    v1 = (rng.random(len(k1)) < 0.85).astype(np.uint8)
    v2 = (rng.random(len(k2)) < 0.85).astype(np.uint8)
    prior = np.full(len(k1), -2, np.int32)
    sel = rng.random(len(k1)) < prior_frac
    prior[sel] = rng.integers(-1, len(k2), sel.sum())
    # relative sim3 of KF1 w.r.t. KF2: x1 = s12 R12 x2 + t12
    R12 = np.eye(3, dtype=np.float32)
    t12 = (-t2).astype(np.float32)
    return (pd.view(k1, d1), pd.view(k2, d2), m1, v1, m2, v2, T1, T2, np.float32(1.0), R12, t12, prior,
            (k1, d1, k2, d2))


def test_fuse_finds_the_shifted_keypoints():
    k1, d1, k2, d2, du, dv = pd.keyframes()
    rng = np.random.default_rng(0)
    T2 = pd.pose_T([du * pd.Z0 / pd.CAM[0], dv * pd.Z0 / pd.CAM[1], 0.0])
    mps = pd.mappoints(k1, d1, pd.pose_T([0, 0, 0]), rng, jitter=0.0, flip=0.0)
    bi, bd = ref_fuse(pd.view(k2, d2), mps, T2, 0)
    ok = bd <= 50
    assert ok.sum() > 300
    # accepted candidates sit where the shifted keypoint is
    assert np.median(np.abs(k2["x"][bi[ok]] - (k1["x"][ok] + du))) < 1.5


def test_sim3_scale_invariance_of_fuse_scw():
    k1, d1, k2, d2, du, dv = pd.keyframes()
    rng = np.random.default_rng(1)
    T2 = pd.pose_T([du * pd.Z0 / pd.CAM[0], dv * pd.Z0 / pd.CAM[1], 0.0])
    mps = pd.mappoints(k1, d1, pd.pose_T([0, 0, 0]), rng)
    S = T2.copy()
    S[:3, :] *= np.float32(2.0)      # Scw = s [R | t], s = 2 (exact in float)
    a = ref_fuse(pd.view(k2, d2), mps, T2, 0)
    b = ref_fuse(pd.view(k2, d2), mps, S, 1)
    assert (a[0] == b[0]).mean() > 0.99


def test_sim3_agreement_finds_matches():
    c = sim3_case()
    new, n = ref_sim3(*c[:12])
    assert n > 100 and n == int((new >= 0).sum())
    prior = c[11]
    assert (new[prior != -2] == -1).all()


def test_distinctive_descriptor_is_the_medoid():
    p, d = pd.distinctive_sets(n_mp=50, seed=3)
    best = ref_distinctive(p, d)
    for m in range(50):
        N = p[m + 1] - p[m]
        if N == 0:
            assert best[m] == -1
            continue
        X = np.unpackbits(d[p[m]:p[m + 1]], axis=1)
        D = (X[:, None, :] != X[None, :, :]).sum(2)
        med = np.sort(D, 1)[:, (N - 1) // 2]
        assert best[m] == int(np.argmin(med))


def ref_proj_kf_sim3(KF, mps, skip, Scw, th, matched):
    L = load()
    L.orbx_ref_search_by_projection_kf_sim3.argtypes = ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int] +
                                                        [ctypes.c_void_p] * 7 + [ctypes.c_int, ctypes.c_void_p,
                                                                                 ctypes.c_void_p])
    out = matched.copy()
    n = ctypes.c_int()
    a = mps[1]
    assert L.orbx_ref_search_by_projection_kf_sim3(ctypes.byref(KF), ptr(pd.CAM), mps[0].n, ptr(a["pos"]),
                                                   ptr(a["normal"]), ptr(a["min_dist"]), ptr(a["max_dist"]),
                                                   ptr(a["desc"]), ptr(skip), ptr(Scw), th, ptr(out),
                                                   ctypes.byref(n)) == 0
    return out, n.value


def ref_proj_frame_kf(F, KF, kf_mps, kf_valid, assigned, Tcw, th, orb_dist, check_ori):
    L = load()
    L.orbx_ref_search_by_projection_frame_kf.argtypes = ([ctypes.c_void_p] * 9 + [ctypes.c_float, ctypes.c_int,
                                                                                 ctypes.c_int, ctypes.c_void_p,
                                                                                 ctypes.c_void_p])
    out = np.zeros(F.n, np.int32)
    n = ctypes.c_int()
    a = kf_mps[1]
    assert L.orbx_ref_search_by_projection_frame_kf(ctypes.byref(F), ctypes.byref(KF), ptr(pd.CAM), ptr(a["pos"]),
                                                    ptr(a["min_dist"]), ptr(a["desc"]), ptr(kf_valid),
                                                    ptr(assigned), ptr(Tcw), th, orb_dist, check_ori, ptr(out),
                                                    ctypes.byref(n)) == 0
    return out, n.value


def seq_case(seed=0):
    k1, d1, k2, d2, du, dv = pd.keyframes()
    rng = np.random.default_rng(seed)
    T2 = pd.pose_T([du * pd.Z0 / pd.CAM[0], dv * pd.Z0 / pd.CAM[1], 0.0])
    mps = pd.mappoints(k1, d1, pd.pose_T([0, 0, 0]), rng)
    return k1, d1, k2, d2, T2, mps, rng


def test_search_by_projection_kf_sim3_assigns_each_keypoint_once():
    k1, d1, k2, d2, T2, mps, rng = seq_case()
    S = T2.copy()
    S[:3, :] *= np.float32(1.5)
    skip = (rng.random(len(k1)) < 0.1).astype(np.uint8)
    matched = np.full(len(k2), -1, np.int32)
    matched[rng.random(len(k2)) < 0.05] = 10 ** 6
    out, n = ref_proj_kf_sim3(pd.view(k2, d2), mps, skip, S, 10, matched)
    new = out[(out >= 0) & (out < 10 ** 6)]
    assert n == len(new) > 200 and len(np.unique(new)) == len(new)
    assert (out[matched == 10 ** 6] == 10 ** 6).all()


def test_search_by_projection_frame_kf_relocalisation():
    k1, d1, k2, d2, T2, mps, rng = seq_case(1)
    valid = (rng.random(len(k1)) < 0.8).astype(np.uint8)
    assigned = (rng.random(len(k2)) < 0.1).astype(np.uint8)
    out, n = ref_proj_frame_kf(pd.view(k2, d2), pd.view(k1, d1), mps, valid, assigned, T2, 10.0, 100, 1)
    assert n == int((out >= 0).sum()) > 200
    assert (out[assigned == 1] == -1).all()
