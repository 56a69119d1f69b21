"""Independent numpy restatements of the vocabulary-node searches
ORBmatcher::SearchByBoW(KeyFrame*, Frame&) (src/ORBmatcher.cc:155-283),
SearchByBoW(KeyFrame*, KeyFrame*) (:715-830) and SearchForTriangulation
with CheckDistEpipolarLine (:852-1014, :136-153), against the oracle's
restatements (oracle/ref_bow.cpp) on the synthetic keyframe pairs of
tests/bow_data.py.

* the FeatureVector walk visits the node ids the two vectors share, in
  ascending order (the lower_bound jumps of the reference skip the others);
  inside a node, features in FeatureVector order;
* KF features need a good map point (state 1; 0 = none, 2 = bad); (KF, F):
  F features already matched in this call are skipped; (KF1, KF2): KF2
  features need a good map point and not to be matched yet;
* best = first minimum, second = second smallest of the candidates'
  distances; (KF, F) accepts best <= TH_LOW, (KF1, KF2) best < TH_LOW, both
  with (float) best < nnratio * (float) second;
* the rotation histogram (angle of the KF / KF1 keypoint minus the other's,
  + 360 when negative, bin = round(rot / 30)) keeps its three largest bins
  (ComputeThreeMaxima's 10 % rule);
* SearchForTriangulation: features without a map point (any state but 0
  counts as one) on both sides, KF2 features not matched yet; candidates at
  distance <= TH_LOW sorted by (distance, index); the first within round(2
  best) whose epipolar distance passes -- the float line a, b, c = x1^T F12,
  num = a x2 + b y2 + c, dsqr = num^2 / (a^2 + b^2) < 3.84 sigma2[octave2]
  in double, den = 0 failing -- is taken; same rotation histogram (KF1 index).
"""
import ctypes

import numpy as np
import pytest

from bow_data import make_pair
from oracle_lib import load
from test_match_numpy import HISTO, hamming, three_maxima

F32 = np.float32
TH_LOW = 50
INT_MAX = 2147483647


def nodes(a):
    ids, ptr, feat = a["ids"], a["ptr"], a["feat"]
    return {int(ids[k]): [int(f) for f in feat[ptr[k]:ptr[k + 1]]] for k in range(len(ids))}


def rot_bin(a1, a2):
    rot = F32(F32(a1) - F32(a2))
    if rot < 0:
        rot = F32(rot + F32(360.0))
    b = int(np.floor(F32(rot * F32(F32(1.0) / F32(HISTO))) + 0.5))
    return 0 if b == HISTO else b


def best_two(d, cand_desc):
    dist = hamming(d, cand_desc)
    b = int(np.argmin(dist))
    second = int(np.sort(dist)[1]) if len(dist) > 1 else INT_MAX
    return b, int(dist[b]), second


def search_by_bow(a1, a2, nnratio, check_ori, kf_kf):
    """kf_kf False: (KF = a1, F = a2), result per F feature (the KF feature
    or -1); True: (KF1 = a1, KF2 = a2), result per KF1 feature."""
    n1, n2 = a1["kps"], a2["kps"]
    out = np.full(len(n2) if not kf_kf else len(n1), -1, np.int64)
    matched2 = np.zeros(len(n2), bool)
    hist = [[] for _ in range(HISTO)]
    nm = 0
    v1, v2 = nodes(a1), nodes(a2)
    for node in sorted(set(v1) & set(v2)):
        for i1 in v1[node]:
            if a1["mp"][i1] != 1:
                continue
            if kf_kf:
                cand = [i2 for i2 in v2[node] if not matched2[i2] and a2["mp"][i2] == 1]
            else:
                cand = [i2 for i2 in v2[node] if not matched2[i2]]
            if not cand:
                continue
            b, best, second = best_two(a1["desc"][i1], a2["desc"][np.array(cand)])
            ok = best < TH_LOW if kf_kf else best <= TH_LOW
            if ok and F32(best) < F32(F32(nnratio) * F32(second)):
                i2 = cand[b]
                matched2[i2] = True
                key = i1 if kf_kf else i2
                out[key] = i2 if kf_kf else i1
                if check_ori:
                    hist[rot_bin(n1["angle"][i1], n2["angle"][i2])].append(key)
                nm += 1
    if check_ori:
        keep = three_maxima(hist)
        for bi in range(HISTO):
            if bi in keep:
                continue
            for key in hist[bi]:
                out[key] = -1
                nm -= 1
    return out, nm


def run_ref(P, mode, nnratio, check_ori):
    L = load()
    V1, V2 = P["V1"], P["V2"]
    out = np.zeros(V2.n if mode == 0 else V1.n, np.int32)
    n = ctypes.c_int()
    fn = "orbx_ref_search_by_bow_frame" if mode == 0 else "orbx_ref_search_by_bow_kf"
    getattr(L, fn).restype = ctypes.c_int
    assert getattr(L, fn)(ctypes.byref(V1), ctypes.byref(V2), ctypes.c_float(nnratio), check_ori,
                          out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n)) == 0
    return out, n.value


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("seed,nnratio,ori,kw", [(0, 0.75, 1, {}), (1, 0.6, 0, {}),
                                                 (2, 0.75, 1, dict(n_nodes=12)),
                                                 (3, 0.9, 1, dict(n1=400, n2=700, same_node=0.6))])
def test_search_by_bow_matches_oracle(mode, seed, nnratio, ori, kw):
    P = make_pair(seed=seed, **kw)
    a1, a2 = P["keep"]
    got, n = search_by_bow(a1, a2, nnratio, ori, kf_kf=mode == 1)
    want, nw = run_ref(P, mode, nnratio, ori)
    assert n == nw and n > 20
    assert np.array_equal(got, want.astype(np.int64))


def epipolar_ok(k1, k2, F, sigma2):
    F = F.reshape(3, 3)
    x1, y1, x2, y2 = F32(k1["x"]), F32(k1["y"]), F32(k2["x"]), F32(k2["y"])
    a = F32(F32(F32(x1 * F[0, 0]) + F32(y1 * F[1, 0])) + F[2, 0])
    b = F32(F32(F32(x1 * F[0, 1]) + F32(y1 * F[1, 1])) + F[2, 1])
    c = F32(F32(F32(x1 * F[0, 2]) + F32(y1 * F[1, 2])) + F[2, 2])
    num = F32(F32(F32(a * x2) + F32(b * y2)) + c)
    den = F32(F32(a * a) + F32(b * b))
    if den == 0:
        return False
    dsqr = F32(F32(num * num) / den)
    return float(dsqr) < 3.84 * float(sigma2[int(k2["octave"])])


def search_for_triangulation(a1, a2, F12, sigma2, check_ori):
    n1, n2 = a1["kps"], a2["kps"]
    out = np.full(len(n1), -1, np.int64)
    matched2 = np.zeros(len(n2), bool)
    hist = [[] for _ in range(HISTO)]
    nm = 0
    v1, v2 = nodes(a1), nodes(a2)
    for node in sorted(set(v1) & set(v2)):
        for i1 in v1[node]:
            if a1["mp"][i1] != 0:
                continue
            cand = [i2 for i2 in v2[node] if not matched2[i2] and a2["mp"][i2] == 0]
            if not cand:
                continue
            dist = hamming(a1["desc"][i1], a2["desc"][np.array(cand)])
            pairs = sorted((int(d), i2) for d, i2 in zip(dist, cand) if d <= TH_LOW)
            if not pairs:
                continue
            th = int(np.floor(2 * pairs[0][0] + 0.5))
            for d, i2 in pairs:
                if d > th:
                    break
                if epipolar_ok(n1[i1], n2[i2], F12, sigma2):
                    matched2[i2] = True
                    out[i1] = i2
                    nm += 1
                    if check_ori:
                        hist[rot_bin(n1["angle"][i1], n2["angle"][i2])].append(i1)
                    break
    if check_ori:
        keep = three_maxima(hist)
        for bi in range(HISTO):
            if bi in keep:
                continue
            for i1 in hist[bi]:
                out[i1] = -1
                nm -= 1
    return out, nm


@pytest.mark.parametrize("seed,ori,kw", [(0, 1, {}), (4, 0, {}), (5, 1, dict(n_nodes=15, mp_probs=(0.7, 0.2, 0.1)))])
def test_search_for_triangulation_matches_oracle(seed, ori, kw):
    P = make_pair(seed=seed, **kw)
    a1, a2 = P["keep"]
    got, n = search_for_triangulation(a1, a2, P["F12"], P["sigma2"], ori)
    L = load()
    out = np.zeros(P["V1"].n, np.int32)
    nr = ctypes.c_int()
    L.orbx_ref_search_for_triangulation.restype = ctypes.c_int
    assert L.orbx_ref_search_for_triangulation(ctypes.byref(P["V1"]), ctypes.byref(P["V2"]),
                                               P["F12"].ctypes.data_as(ctypes.c_void_p),
                                               P["sigma2"].ctypes.data_as(ctypes.c_void_p), ori,
                                               out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nr)) == 0
    assert n == nr.value and n > 20
    assert np.array_equal(got, out.astype(np.int64))
