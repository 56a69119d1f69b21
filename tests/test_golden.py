"""Golden vectors (tests/golden/*.npz, made by tools/gen_golden.py).

CPU tests: the oracle still reproduces every committed vector (catches any
drift of the restatement).  GPU tests: the product (liborbx through the C
ABI) reproduces the same vectors from data alone -- bit-exact for
extraction and matching, 1e-5 on poses for local BA (north_star tolerance).
"""
import ctypes
from pathlib import Path

import numpy as np
import pytest

import orb_slam_amd as ox
from orb_slam_amd import synth_ba as sb
from oracle_lib import KEYPOINT, RefExtractor, load, ptr

GOLD = Path(__file__).resolve().parent / "golden"
# each image in both libstdc++ eras of retainBest: `<name>` GCC 4.6 .. 4.8
# (the default), `<name>_gcc49` GCC >= 4.9 (tools/gen_golden.py ERAS)
EXTRACT = [n + s for n in ("extract_texture_320x240", "extract_noise_160x120", "extract_ragged_97x71")
           for s in ("", "_gcc49")]


def era(z):
    return int(z["nth_pivot"])


def g(name):
    return np.load(GOLD / f"{name}.npz")


def kps(a):
    return np.ascontiguousarray(a).view(KEYPOINT).reshape(-1)


def lba_problem(z):
    prob = {k[3:]: z[k] for k in z.files if k.startswith("in_")}
    prob["huber_delta"] = float(z["huber_delta"])
    prob["chi2_threshold"] = float(z["chi2_threshold"])
    return prob


# ------------------------------------------------------------------ oracle
@pytest.mark.parametrize("name", EXTRACT)
def test_oracle_extract_golden(name):
    z = g(name)
    k, d = RefExtractor(int(z["nfeatures"]), nth_pivot=era(z))(z["image"])
    assert np.array_equal(k.view(np.uint8).reshape(-1, 28), z["keypoints"])
    assert np.array_equal(d, z["descriptors"])


def test_golden_eras_differ():
    """The two eras' vectors of each image differ (so both are pinned)."""
    for n in EXTRACT[::2]:
        assert not np.array_equal(g(n)["keypoints"], g(n + "_gcc49")["keypoints"]), n


def test_oracle_search_init_golden():
    z = g("search_init_320x240")
    k1, k2 = kps(z["kps1"]), kps(z["kps2"])
    d1, d2 = np.ascontiguousarray(z["desc1"]), np.ascontiguousarray(z["desc2"])
    F1, F2 = ox.frame_view(k1, d1, int(z["w"]), int(z["h"])), ox.frame_view(k2, d2, int(z["w"]), int(z["h"]))
    prev = z["prev_in"].copy()
    m = np.zeros(len(k1), np.int32)
    n = ctypes.c_int()
    assert load().orbx_ref_search_for_initialization(ctypes.byref(F1), ctypes.byref(F2), ptr(prev), ptr(m),
                                                     int(z["window"]), float(z["nnratio"]), int(z["check_ori"]),
                                                     ctypes.byref(n)) == 0
    assert n.value == int(z["n_matches"])
    assert np.array_equal(m, z["matches12"]) and np.array_equal(prev, z["prev_out"])


def test_oracle_hamming_golden():
    z = g("hamming_bf")
    a, b = np.ascontiguousarray(z["desc_a"]), np.ascontiguousarray(z["desc_b"])
    bi, best, sec = (np.zeros(len(a), np.int32) for _ in range(3))
    load().orbx_ref_hamming_bf(ptr(a), len(a), ptr(b), len(b), ptr(bi), ptr(best), ptr(sec))
    assert np.array_equal(bi, z["best_idx"]) and np.array_equal(best, z["best"]) and np.array_equal(sec, z["second"])
    # size-independent properties: best is the minimum, second >= best
    dist = np.unpackbits(a[:, None, :] ^ b[None, :, :], axis=2).sum(2)
    assert np.array_equal(best, dist.min(1)) and (sec >= best).all()
    assert np.array_equal(bi, dist.argmin(1))       # first index among ties


def test_oracle_lba_golden():
    z = g("lba_small")
    p, arrs = sb.to_ctypes(lba_problem(z))
    es = np.zeros(p.n_edges, np.uint8)
    pb = np.zeros(p.n_points, np.uint8)
    st = sb.BAStats()
    L = load()
    L.orbx_ref_lba.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p]
    assert L.orbx_ref_lba(ctypes.byref(p), int(z["iters0"]), int(z["iters1"]), ptr(es), ptr(pb),
                          ctypes.byref(st)) == 0
    assert np.abs(arrs["pose_q"] - z["out_pose_q"]).max() < 1e-9
    assert np.abs(arrs["pose_t"] - z["out_pose_t"]).max() < 1e-9
    assert np.array_equal(es, z["edge_status"]) and np.array_equal(pb, z["point_bad"])
    assert list(st.iterations) == list(z["iterations"])


# ------------------------------------------------------------------ product
@pytest.fixture(scope="module")
def gctx():
    c = ox.Context(nfeatures=500, max_w=320, max_h=240, slots=1)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", EXTRACT)
def test_gpu_extract_golden(name):
    z = g(name)
    img = z["image"]
    c = ox.Context(nfeatures=int(z["nfeatures"]), max_w=img.shape[1], max_h=img.shape[0], slots=1)
    try:
        if era(z) != 1:   # 1 is the default
            c.set_nth_pivot(era(z))
        k, d = c(img)
    finally:
        c.close()
    assert np.array_equal(k.view(np.uint8).reshape(-1, 28), z["keypoints"])
    assert np.array_equal(d, z["descriptors"])


@pytest.mark.gpu
def test_gpu_search_init_golden(gctx):
    z = g("search_init_320x240")
    k1, k2 = kps(z["kps1"]), kps(z["kps2"])
    d1, d2 = np.ascontiguousarray(z["desc1"]), np.ascontiguousarray(z["desc2"])
    F1, F2 = ox.frame_view(k1, d1, int(z["w"]), int(z["h"])), ox.frame_view(k2, d2, int(z["w"]), int(z["h"]))
    prev = z["prev_in"].copy()
    m = np.zeros(len(k1), np.int32)
    n = ctypes.c_int()
    assert ox.lib().orbx_search_for_initialization(gctx.handle, ctypes.byref(F1), ctypes.byref(F2), ox._ptr(prev),
                                                   ox._ptr(m), int(z["window"]), float(z["nnratio"]),
                                                   int(z["check_ori"]), ctypes.byref(n)) == 0
    assert n.value == int(z["n_matches"])
    assert np.array_equal(m, z["matches12"]) and np.array_equal(prev, z["prev_out"])


@pytest.mark.gpu
def test_gpu_hamming_golden(gctx):
    z = g("hamming_bf")
    a, b = np.ascontiguousarray(z["desc_a"]), np.ascontiguousarray(z["desc_b"])
    bi, best, sec = (np.zeros(len(a), np.int32) for _ in range(3))
    assert ox.lib().orbx_hamming_bf(gctx.handle, ox._ptr(a), len(a), ox._ptr(b), len(b), ox._ptr(bi), ox._ptr(best),
                                    ox._ptr(sec)) == 0
    assert np.array_equal(bi, z["best_idx"]) and np.array_equal(best, z["best"]) and np.array_equal(sec, z["second"])


@pytest.mark.gpu
def test_gpu_lba_golden(gctx):
    z = g("lba_small")
    p, arrs = sb.to_ctypes(lba_problem(z))
    es = np.zeros(p.n_edges, np.uint8)
    pb = np.zeros(p.n_points, np.uint8)
    st = sb.BAStats()
    assert ox.lib().orbx_lba_solve(gctx.handle, ctypes.byref(p), int(z["iters0"]), int(z["iters1"]), None,
                                   es.ctypes.data, pb.ctypes.data, ctypes.byref(st)) == 0
    assert np.abs(arrs["pose_q"] - z["out_pose_q"]).max() <= 1e-5
    assert np.abs(arrs["pose_t"] - z["out_pose_t"]).max() <= 1e-5
    assert np.abs(arrs["points"] - z["out_points"]).max() <= 1e-4
    assert np.array_equal(es, z["edge_status"]) and np.array_equal(pb, z["point_bad"])
    assert list(st.iterations) == list(z["iterations"])


# ------------------------------------------------------------------ pose optimisation
def pose_frame(z):
    return {k[3:]: z[k].copy() for k in z.files if k.startswith("in_")}


def test_oracle_pose_golden():
    from orb_slam_amd import synth_pose as sp
    z = g("pose_frame")
    p, arrs = sp.to_ctypes(pose_frame(z))
    n = ctypes.c_int()
    st = sp.PoseStats()
    L = load()
    L.orbx_ref_pose_optimization.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    assert L.orbx_ref_pose_optimization(ctypes.byref(p), ctypes.byref(n), ctypes.byref(st)) == 0
    assert np.array_equal(sp.pose_of(p), z["out_Tcw"])
    assert np.array_equal(arrs["outlier"], z["out_outlier"]) and n.value == int(z["n_inliers"])
    assert list(st.iterations) == list(z["iterations"]) and list(st.n_bad) == list(z["n_bad"])


@pytest.mark.gpu
def test_gpu_pose_golden(gctx):
    from orb_slam_amd import synth_pose as sp
    z = g("pose_frame")
    p, arrs = sp.to_ctypes(pose_frame(z))
    n, st = gctx.pose_optimization([p])
    assert np.abs(sp.pose_of(p) - z["out_Tcw"]).max() <= 1e-5
    assert np.array_equal(arrs["outlier"], z["out_outlier"]) and int(n[0]) == int(z["n_inliers"])
    assert st[0].rounds == int(z["rounds"]) and list(st[0].n_bad) == list(z["n_bad"])


# ------------------------------------------------------------------ vocabulary-node searches, DBoW2 transform
def bow_views(z):
    from bow_data import make_view
    out = []
    for tag in ("a", "b"):
        kps = np.ascontiguousarray(z[f"{tag}_kps"]).view(ox.KEYPOINT).reshape(-1)
        ids, ptr_, feat = z[f"{tag}_ids"], z[f"{tag}_ptr"], z[f"{tag}_feat"]
        node_of = np.zeros(len(kps), np.int64)
        for j in range(len(ids)):
            node_of[feat[ptr_[j]:ptr_[j + 1]]] = ids[j]
        out.append(make_view(kps, z[f"{tag}_desc"], z[f"{tag}_mp"], node_of))
    return out


def bow_pair(z):
    (V1, a1), (V2, a2) = bow_views(z)
    return {"V1": V1, "V2": V2, "keep": (a1, a2), "F12": z["F12"].copy(), "sigma2": z["sigma2"].copy()}


def test_oracle_bow_golden():
    from test_bow_oracle import run_ref
    z = g("bow_pair")
    P = bow_pair(z)
    for mode, name in [(0, "bow_frame"), (1, "bow_kf"), (2, "triangulation")]:
        m, n = run_ref(mode, P, 0.75, 1)
        assert n == int(z[f"{name}_n"]) and np.array_equal(m, z[f"{name}_matches"])


@pytest.mark.gpu
def test_gpu_bow_golden(gctx):
    from test_bow_gpu import run_gpu
    z = g("bow_pair")
    P = bow_pair(z)
    for mode, name in [(0, "bow_frame"), (1, "bow_kf"), (2, "triangulation")]:
        m, n = run_gpu(gctx, mode, P, 0.75, 1)
        assert n == int(z[f"{name}_n"]) and np.array_equal(m, z[f"{name}_matches"])


def vocab_from(z):
    return {"k": int(z["k"]), "L": int(z["L"]), "parent": z["parent"].copy(), "is_leaf": z["is_leaf"].copy(),
            "desc": np.ascontiguousarray(z["vdesc"]), "weight": z["weight"].copy()}


def check_vocab(z, r):
    nw, nf = len(z["bow_words"]), len(z["fv_nodes"])
    assert np.array_equal(r["word"], z["word"]) and np.array_equal(r["weight"], z["w"])
    assert np.array_equal(r["nid"], z["nid"]) and r["nw"] == nw and r["nf"] == nf
    assert np.array_equal(r["bw"][:nw], z["bow_words"]) and np.array_equal(r["bv"][:nw], z["bow_values"])
    assert np.array_equal(r["fn"][:nf], z["fv_nodes"]) and np.array_equal(r["fp"][:nf + 1], z["fv_ptr"])
    assert np.array_equal(r["ff"][:len(z["fv_feat"])], z["fv_feat"])


def test_oracle_vocab_golden():
    from vocab_data import run_ref
    z = g("vocab_small")
    check_vocab(z, run_ref(vocab_from(z), np.ascontiguousarray(z["desc"]), int(z["levelsup"])))


@pytest.mark.gpu
def test_gpu_vocab_golden(gctx):
    from test_vocab_gpu import gpu_transform
    z = g("vocab_small")
    check_vocab(z, gpu_transform(gctx, vocab_from(z), np.ascontiguousarray(z["desc"]), int(z["levelsup"])))
