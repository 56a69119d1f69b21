"""Independent numpy restatements of the vocabulary-node searches
ORBmatcher::SearchByBoW(KeyFrame*, Frame&) (src/ORBmatcher.cc:155-283) and
SearchByBoW(KeyFrame*, KeyFrame*) (:715-830), against the oracle's
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
  (ComputeThreeMaxima's 10 % rule).
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
