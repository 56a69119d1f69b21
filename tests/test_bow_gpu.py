"""GPU vocabulary-node searches through the C ABI against the CPU
restatement (oracle/ref_bow.cpp): SearchByBoW(KF, F) (src/ORBmatcher.cc:
155-283), SearchByBoW(KF1, KF2) (:715-850), SearchForTriangulation
(:852-1014).  Match vectors and counts must be identical."""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
from bow_data import make_pair
from test_bow_oracle import run_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
    yield c
    c.close()


def run_gpu(ctx, mode, P, nnratio=0.75, check_ori=1):
    V1, V2 = P["V1"], P["V2"]
    out = np.zeros(V2.n if mode == 0 else V1.n, np.int32)
    n = ctypes.c_int()
    L = ox.lib()
    if mode == 0:
        r = L.orbx_search_by_bow_frame(ctx.handle, ctypes.byref(V1), ctypes.byref(V2), nnratio, check_ori,
                                       ox._ptr(out), ctypes.byref(n))
    elif mode == 1:
        r = L.orbx_search_by_bow_kf(ctx.handle, ctypes.byref(V1), ctypes.byref(V2), nnratio, check_ori,
                                    ox._ptr(out), ctypes.byref(n))
    else:
        r = L.orbx_search_for_triangulation(ctx.handle, ctypes.byref(V1), ctypes.byref(V2), ox._ptr(P["F12"]),
                                            ox._ptr(P["sigma2"]), 8, check_ori, ox._ptr(out), ctypes.byref(n))
    assert r == 0, r
    return out, n.value


CASES = [dict(seed=0), dict(seed=1, n_nodes=20), dict(seed=2, n_nodes=3), dict(seed=3, n1=300, n2=1500),
         dict(seed=4, n_nodes=1, n1=400, n2=2000), dict(seed=6, match_frac=0.9, mp_probs=(0.2, 0.7, 0.1))]


@pytest.mark.parametrize("mode", [0, 1, 2], ids=["bow_frame", "bow_kf", "triangulation"])
@pytest.mark.parametrize("case", CASES, ids=[f"s{c['seed']}" for c in CASES])
@pytest.mark.parametrize("check_ori,nnratio", [(1, 0.75), (0, 0.9)])
def test_bow_matches_oracle(ctx, mode, case, check_ori, nnratio):
    P = make_pair(**case)
    ro, rn = run_ref(mode, P, nnratio, check_ori)
    go, gn = run_gpu(ctx, mode, P, nnratio, check_ori)
    assert gn == rn and rn > 0
    assert np.array_equal(go, ro), np.count_nonzero(go != ro)


def test_bow_empty_and_disjoint(ctx):
    P = make_pair(seed=7, n1=50, n2=0)
    for mode in (0, 1, 2):
        go, gn = run_gpu(ctx, mode, P)
        ro, rn = run_ref(mode, P)
        assert gn == rn == 0 and np.array_equal(go, ro)
    A = make_pair(seed=8, node_pool=np.arange(0, 50))
    B = make_pair(seed=9, node_pool=np.arange(100, 150))
    P = {"V1": A["V1"], "V2": B["V2"], "keep": (A["keep"], B["keep"]), "F12": A["F12"], "sigma2": A["sigma2"]}
    for mode in (0, 1, 2):
        go, gn = run_gpu(ctx, mode, P)
        assert gn == 0 and (go == -1).all()


def test_bow_rejects_duplicate_feature(ctx):
    P = make_pair(seed=10, n1=100, n2=100)
    a1 = P["keep"][0]
    a1["feat"][1] = a1["feat"][0]          # a feature listed in two places
    out = np.zeros(100, np.int32)
    n = ctypes.c_int()
    assert ox.lib().orbx_search_by_bow_kf(ctx.handle, ctypes.byref(P["V1"]), ctypes.byref(P["V2"]), 0.75, 1,
                                          ox._ptr(out), ctypes.byref(n)) == -1
