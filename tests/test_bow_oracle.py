"""CPU checks of the vocabulary-node search restatements (oracle/ref_bow.cpp;
src/ORBmatcher.cc:155-283, 715-1014): known answers on hand-built cases and
invariants on the synthetic pairs the GPU parity tests use."""
import ctypes

import numpy as np

import orb_slam_amd as ox
from bow_data import make_pair, make_view
from oracle_lib import load


def ref(fn, *args):
    L = load()
    getattr(L, fn).restype = ctypes.c_int
    return getattr(L, fn)(*args)


def run_ref(mode, P, nnratio=0.75, check_ori=1):
    V1, V2 = P["V1"], P["V2"]
    out = np.zeros(V2.n if mode == 0 else V1.n, np.int32)
    n = ctypes.c_int()
    if mode == 0:
        assert ref("orbx_ref_search_by_bow_frame", ctypes.byref(V1), ctypes.byref(V2), ctypes.c_float(nnratio),
                   check_ori, out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n)) == 0
    elif mode == 1:
        assert ref("orbx_ref_search_by_bow_kf", ctypes.byref(V1), ctypes.byref(V2), ctypes.c_float(nnratio),
                   check_ori, out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n)) == 0
    else:
        assert ref("orbx_ref_search_for_triangulation", ctypes.byref(V1), ctypes.byref(V2),
                   P["F12"].ctypes.data_as(ctypes.c_void_p), P["sigma2"].ctypes.data_as(ctypes.c_void_p), check_ori,
                   out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n)) == 0
    return out, n.value


def tiny(desc2_bits, mp1=1, mp2=1, node2=7):
    k = np.zeros(2, ox.KEYPOINT)
    k["x"], k["y"], k["angle"] = [100.0, 200.0], [100.0, 150.0], [10.0, 10.0]
    d1 = np.zeros((2, 32), np.uint8)
    d1[1, :] = 0xFF
    d2 = d1.copy()
    d2[0, 0] ^= desc2_bits
    A, aa = make_view(k, d1, np.array([mp1, mp1], np.uint8), np.array([7, 9]))
    B, ab = make_view(k.copy(), d2, np.array([mp2, mp2], np.uint8), np.array([node2, 9]))
    return {"V1": A, "V2": B, "keep": (aa, ab), "F12": np.zeros(9, np.float32), "sigma2": np.ones(8, np.float32)}


def test_identical_descriptors_match_in_shared_nodes():
    P = tiny(0)
    out, n = run_ref(1, P, nnratio=0.9)
    assert n == 2 and list(out) == [0, 1]
    out, n = run_ref(0, P, nnratio=0.9)
    assert n == 2 and list(out) == [0, 1]


def test_different_nodes_never_match():
    P = tiny(0, node2=8)
    out, n = run_ref(1, P, nnratio=0.9)
    assert n == 1 and list(out) == [-1, 1]


def test_map_point_states_gate_the_searches():
    out, n = run_ref(1, tiny(0, mp2=2), nnratio=0.9)        # bad map points in KF2
    assert n == 0
    out, n = run_ref(0, tiny(0, mp1=0), nnratio=0.9)        # KF without map points
    assert n == 0


def test_th_low_boundary_differs_between_variants():
    # one descriptor 50 bits away: SearchByBoW(KF, F) accepts (<= TH_LOW),
    # SearchByBoW(KF1, KF2) rejects (< TH_LOW)
    k = np.zeros(1, ox.KEYPOINT)
    d1 = np.zeros((1, 32), np.uint8)
    d2 = d1.copy()
    d2[0, :6] = 0xFF
    d2[0, 6] = 0x03          # 50 bits
    A, aa = make_view(k, d1, np.ones(1, np.uint8), np.array([3]))
    B, ab = make_view(k.copy(), d2, np.ones(1, np.uint8), np.array([3]))
    P = {"V1": A, "V2": B, "keep": (aa, ab)}
    assert run_ref(0, P, 0.9, 0)[1] == 1
    assert run_ref(1, P, 0.9, 0)[1] == 0


def test_synthetic_pair_recovers_correspondences():
    P = make_pair(seed=1)
    for mode in (0, 1, 2):
        out, n = run_ref(mode, P)
        assert n == int((out >= 0).sum()) and n > 20, (mode, n)
        # a KF2 feature is matched at most once
        m = out[out >= 0]
        assert len(np.unique(m)) == len(m)
