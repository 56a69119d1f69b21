"""Device-resident BoW of extracted frames through the C ABI against the CPU
restatement: orbx_dev_compute_bow (Frame::ComputeBoW, src/Frame.cc:279-286,
as TemplatedVocabulary::transform, Thirdparty/DBoW2/DBoW2/
TemplatedVocabulary.h:1127-1259) must give the oracle transform's
per-feature results, BowVector (values bit-identical) and FeatureVector;
orbx_dev_search_by_bow (Tracking::Relocalisation's loop, src/Tracking.cc:
904-925, over ORBmatcher::SearchByBoW(KF, F), src/ORBmatcher.cc:155-283)
must give the oracle's match vectors and counts for every candidate."""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
from orb_slam_amd import synth
from bow_data import BowView
from test_bow_oracle import run_ref as ref_search
from vocab_data import make_vocab, run_ref as ref_transform

pytestmark = pytest.mark.gpu

W, H = 640, 480


@pytest.fixture(scope="module")
def ctx():
    c = ox.Context(nfeatures=1000, max_w=W, max_h=H, slots=4)
    yield c
    c.close()


@pytest.fixture(scope="module")
def extracted(ctx):
    frames = synth.sequence(W, H, 3, seed=91)
    ctx.upload(np.stack(frames), 0)
    ctx.upload(synth.texture_frame(W, H, seed=5), 3)
    ctx.extract(0, 4)
    ctx.sync()
    return [ctx.features(s) for s in range(4)]


def create_vocab(ctx, V):
    voc = ctypes.c_void_p()
    assert ox.lib().orbx_vocab_create(ctx.handle, V["k"], V["L"], len(V["parent"]), ox._ptr(V["parent"]),
                                      ox._ptr(V["is_leaf"]), ox._ptr(V["desc"]), ox._ptr(V["weight"]),
                                      ctypes.byref(voc)) == 0
    return voc


def read_bow(ctx, slot, n):
    out = {"word": np.zeros(n, np.int32), "weight": np.zeros(n), "nid": np.zeros(n, np.int32),
           "bw": np.zeros(n, np.uint32), "bv": np.zeros(n), "fn": np.zeros(n, np.uint32),
           "fp": np.zeros(n + 1, np.int32), "ff": np.zeros(n, np.int32)}
    nw, nf = ctypes.c_int(), ctypes.c_int()
    r = ox.lib().orbx_dev_read_bow(ctx.handle, slot, n, ox._ptr(out["word"]), ox._ptr(out["weight"]),
                                   ox._ptr(out["nid"]), ox._ptr(out["bw"]), ox._ptr(out["bv"]), ctypes.byref(nw),
                                   ox._ptr(out["fn"]), ox._ptr(out["fp"]), ox._ptr(out["ff"]), ctypes.byref(nf))
    assert r == 0, r
    out["nw"], out["nf"] = nw.value, nf.value
    return out


def view(kps, desc, mp, T):
    """orbx_bow_view over a frame and its transform result T (FeatureVector CSR)."""
    nn = T["nf"]
    arrs = {"kps": np.ascontiguousarray(kps), "desc": np.ascontiguousarray(desc, np.uint8),
            "mp": np.ascontiguousarray(mp, np.uint8), "ids": T["fn"][:nn].copy(), "ptr": T["fp"][:nn + 1].copy(),
            "feat": T["ff"][:max(int(T["fp"][nn]), 1)].copy()}
    v = BowView()
    v.keys = arrs["kps"].ctypes.data
    v.desc = arrs["desc"].ctypes.data
    v.n = len(kps)
    v.mp = arrs["mp"].ctypes.data
    v.n_nodes = nn
    v.node_id = arrs["ids"].ctypes.data if nn else None
    v.node_ptr = arrs["ptr"].ctypes.data
    v.feat_idx = arrs["feat"].ctypes.data
    return v, arrs


def search(ctx, slot, KFs, nnratio, check_ori, cap=None):
    cap = cap or ctx.nfeatures
    outs = [np.zeros(cap, np.int32) for _ in KFs]
    ptrs = (ctypes.c_void_p * max(len(KFs), 1))(*[o.ctypes.data for o in outs])
    arr = (BowView * max(len(KFs), 1))(*KFs)
    nm = np.zeros(max(len(KFs), 1), np.int32)
    r = ox.lib().orbx_dev_search_by_bow(ctx.handle, slot, len(KFs), arr, nnratio, check_ori, ptrs, cap,
                                        ox._ptr(nm))
    return r, outs, nm[:len(KFs)]


# (k, L, levelsup): FeatureVector at level L - levelsup (100 nodes at level
# 2 as with ORBvoc and levelsup 4; 10 wide nodes at level 1)
VOCABS = [(10, 5, 3), (10, 5, 4), (6, 5, 2)]


@pytest.mark.parametrize("k,L,levelsup", VOCABS)
def test_dev_compute_bow_matches_oracle(ctx, extracted, k, L, levelsup):
    V = make_vocab(k=k, L=L, seed=k + L, irregular=k == 6)
    voc = create_vocab(ctx, V)
    try:
        assert ox.lib().orbx_dev_compute_bow(ctx.handle, voc, 0, 4, levelsup) == 0
        for s in range(4):
            kps, desc = extracted[s]
            n = len(kps)
            assert n > 500
            r = ref_transform(V, desc, levelsup)
            g = read_bow(ctx, s, n)
            for key in ["word", "weight", "nid"]:
                assert np.array_equal(g[key], r[key]), (s, key)
            assert g["nw"] == r["nw"] and g["nf"] == r["nf"]
            assert np.array_equal(g["bw"][:r["nw"]], r["bw"][:r["nw"]])
            assert np.array_equal(g["bv"][:r["nw"]].view(np.uint64), r["bv"][:r["nw"]].view(np.uint64))
            assert np.array_equal(g["fn"][:r["nf"]], r["fn"][:r["nf"]])
            assert np.array_equal(g["fp"][:r["nf"] + 1], r["fp"][:r["nf"] + 1])
            m = int(r["fp"][r["nf"]])
            assert np.array_equal(g["ff"][:m], r["ff"][:m])
    finally:
        ox.lib().orbx_vocab_destroy(voc)


@pytest.mark.parametrize("k,L,levelsup", VOCABS)
@pytest.mark.parametrize("check_ori,nnratio", [(1, 0.75), (0, 0.9)])
def test_dev_search_by_bow_matches_oracle(ctx, extracted, k, L, levelsup, check_ori, nnratio):
    V = make_vocab(k=k, L=L, seed=k + L, irregular=k == 6)
    voc = create_vocab(ctx, V)
    try:
        rng = np.random.default_rng(k * 100 + L * 10 + levelsup)
        assert ox.lib().orbx_dev_compute_bow(ctx.handle, voc, 0, 1, levelsup) == 0
        fk, fd = extracted[0]
        Fv, fa = view(fk, fd, np.zeros(len(fk), np.uint8), ref_transform(V, fd, levelsup))
        # candidates: the next frames of the sequence, an unrelated frame and
        # the frame itself, map-point states random
        KFs, keep = [], []
        for s in (1, 2, 3, 0):
            kk, kd = extracted[s]
            mp = rng.choice(3, len(kk), p=(0.3, 0.6, 0.1)).astype(np.uint8)
            v, a = view(kk, kd, mp, ref_transform(V, kd, levelsup))
            KFs.append(v)
            keep.append(a)
        r, outs, nm = search(ctx, 0, KFs, nnratio, check_ori)
        assert r == 0, r
        for i, KF in enumerate(KFs):
            ro, rn = ref_search(0, {"V1": KF, "V2": Fv}, nnratio, check_ori)
            assert nm[i] == rn, (i, nm[i], rn)
            assert np.array_equal(outs[i][:len(fk)], ro), (i, np.count_nonzero(outs[i][:len(fk)] != ro))
            assert np.all(outs[i][len(fk):] == -1)
        assert nm[3] > 100   # the frame against itself
    finally:
        ox.lib().orbx_vocab_destroy(voc)


def test_dev_bow_state_and_errors(ctx, extracted):
    V = make_vocab(k=10, L=4, seed=3)
    voc = create_vocab(ctx, V)
    try:
        L = ox.lib()
        assert L.orbx_dev_compute_bow(ctx.handle, voc, 0, 2, 2) == 0
        n = len(extracted[1][0])
        read_bow(ctx, 1, n)
        assert L.orbx_dev_read_bow(ctx.handle, 1, n - 1, None, None, None, None, None, None, None, None, None,
                                   None) == -3
        assert L.orbx_dev_compute_bow(ctx.handle, voc, 3, 2, 2) == -1   # past the slots
        assert search(ctx, 0, [], 0.75, 1)[0] == 0                                   # no candidates
        assert search(ctx, 0, [BowView()], 0.75, 1, cap=10)[0] == -3
        # re-extracting a slot drops its BoW until computed again
        ctx.extract(1, 1)
        assert L.orbx_dev_read_bow(ctx.handle, 1, n, None, None, None, None, None, None, None, None, None,
                                   None) == -1
        assert search(ctx, 1, [BowView()], 0.75, 1)[0] == -1
        assert L.orbx_dev_compute_bow(ctx.handle, voc, 1, 1, 2) == 0
        read_bow(ctx, 1, n)
        # an empty keyframe matches nothing
        r, outs, nm = search(ctx, 0, [BowView()], 0.75, 1)
        assert r == 0 and nm[0] == 0 and np.all(outs[0] == -1)
    finally:
        ox.lib().orbx_vocab_destroy(voc)


def search_kf(ctx, mode, slot1, mp1, slots2, mp2s, nnratio=0.75, check_ori=1, F12s=None, sigma2s=None, cap=None):
    cap = cap or ctx.nfeatures
    n = len(slots2)
    outs = [np.zeros(cap, np.int32) for _ in range(n)]
    ptrs = (ctypes.c_void_p * max(n, 1))(*[o.ctypes.data for o in outs])
    mps = (ctypes.c_void_p * max(n, 1))(*[m.ctypes.data for m in mp2s])
    s2 = np.ascontiguousarray(slots2, np.int32)
    nm = np.zeros(max(n, 1), np.int32)
    L = ox.lib()
    if mode == 1:
        r = L.orbx_dev_search_by_bow_kf(ctx.handle, slot1, ox._ptr(mp1), n, ox._ptr(s2), mps, nnratio, check_ori, ptrs,
                                        cap, ox._ptr(nm))
    else:
        r = L.orbx_dev_search_for_triangulation(ctx.handle, slot1, ox._ptr(mp1), n, ox._ptr(s2), mps, ox._ptr(F12s),
                                                ox._ptr(sigma2s), 8, check_ori, ptrs, cap, ox._ptr(nm))
    return r, outs, nm[:n]


def translation_f12(dx, dy):
    """F12 of a pure image translation (dx, dy): the epipolar line of kp1 is
    the line through it along (dx, dy) (a = -dy, b = dx, c = x dy - y dx)."""
    return np.array([0, 0, dy, 0, 0, -dx, -dy, dx, 0], np.float32)


def level_sigma2(nlevels=8, scale=1.2):
    s, out = np.float32(1.0), []
    for _ in range(nlevels):
        out.append(np.float32(s * s))
        s = np.float32(s * np.float32(scale))
    return np.array(out, np.float32)


@pytest.mark.parametrize("k,L,levelsup", VOCABS[:2])
@pytest.mark.parametrize("mode", [1, 2], ids=["bow_kf", "triangulation"])
@pytest.mark.parametrize("check_ori", [1, 0])
def test_dev_kf_searches_match_oracle(ctx, extracted, k, L, levelsup, mode, check_ori):
    V = make_vocab(k=k, L=L, seed=k + L, irregular=False)
    voc = create_vocab(ctx, V)
    try:
        rng = np.random.default_rng(7 * k + L + mode)
        assert ox.lib().orbx_dev_compute_bow(ctx.handle, voc, 0, 4, levelsup) == 0
        probs = (0.3, 0.6, 0.1) if mode == 1 else (0.6, 0.3, 0.1)
        views, mps = [], []
        for s in range(4):
            kk, kd = extracted[s]
            mp = rng.choice(3, len(kk), p=probs).astype(np.uint8)
            views.append(view(kk, kd, mp, ref_transform(V, kd, levelsup)))
            mps.append(mp)
        slots2 = [1, 2, 3, 0]
        F12s = np.concatenate([translation_f12(1.0, 0.3 * s) for s in slots2]).astype(np.float32)
        sig = level_sigma2()
        sigma2s = np.tile(sig, len(slots2)).astype(np.float32)
        r, outs, nm = search_kf(ctx, mode, 0, mps[0], slots2, [mps[s] for s in slots2], 0.75, check_ori, F12s, sigma2s)
        assert r == 0, r
        n1 = len(extracted[0][0])
        for i, s in enumerate(slots2):
            P = {"V1": views[0][0], "V2": views[s][0], "F12": F12s[9 * i:9 * i + 9].copy(), "sigma2": sig}
            ro, rn = ref_search(mode, P, 0.75, check_ori)
            assert nm[i] == rn, (i, nm[i], rn)
            assert np.array_equal(outs[i][:n1], ro), (i, np.count_nonzero(outs[i][:n1] != ro))
            assert np.all(outs[i][n1:] == -1)
        assert nm[3] > 50   # slot 0 against itself
    finally:
        ox.lib().orbx_vocab_destroy(voc)


def test_dev_kf_search_errors(ctx, extracted):
    V = make_vocab(k=10, L=4, seed=3)
    voc = create_vocab(ctx, V)
    try:
        L = ox.lib()
        mp = np.ones(ctx.nfeatures, np.uint8)
        assert L.orbx_dev_compute_bow(ctx.handle, voc, 0, 2, 2) == 0
        assert search_kf(ctx, 1, 0, mp, [], [])[0] == 0
        assert search_kf(ctx, 1, 0, mp, [1], [mp], cap=10)[0] == -3
        ctx.extract(2, 2)                                   # slots 2, 3: no BoW
        assert search_kf(ctx, 1, 0, mp, [2], [mp])[0] == -1
        assert search_kf(ctx, 1, 0, mp, [4], [mp])[0] == -1   # no such slot
        r, outs, nm = search_kf(ctx, 1, 0, mp, [1], [mp])
        assert r == 0 and nm[0] > 0
        F = translation_f12(1.0, 0.0)
        assert search_kf(ctx, 2, 0, mp, [1], [mp], F12s=F, sigma2s=level_sigma2(9))[0] == 0
        assert ox.lib().orbx_dev_search_for_triangulation(ctx.handle, 0, ox._ptr(mp), 1,
                                                          ox._ptr(np.array([1], np.int32)),
                                                          (ctypes.c_void_p * 1)(mp.ctypes.data), ox._ptr(F),
                                                          ox._ptr(level_sigma2(7)), 7, 1,
                                                          (ctypes.c_void_p * 1)(outs[0].ctypes.data), 1000,
                                                          ox._ptr(nm)) == -1   # nlevels != the extractor's
        assert L.orbx_dev_compute_bow(ctx.handle, voc, 2, 2, 2) == 0
    finally:
        ox.lib().orbx_vocab_destroy(voc)


def test_dev_bow_after_async_pipeline():
    """orbx_dev_compute_bow right after an asynchronous, three-part
    extract_match (no sync in between) sees the finished extraction: the BoW
    of every slot equals the oracle transform of the slot's descriptors, and
    a Relocalisation search over the batch's frames equals the oracle's."""
    B = 48   # three pipeline parts
    c = ox.Context(nfeatures=1000, max_w=W, max_h=H, slots=2 * B)
    try:
        V = make_vocab(k=10, L=5, seed=15)
        voc = create_vocab(c, V)
        frames = np.stack(synth.sequence(W, H, B, seed=123))
        c.upload(frames, 0)
        c.upload(frames[::-1].copy(), B)
        c.set_async_match(True)
        c.extract_match(0, B, B)
        c.extract_match(B, B, B)          # the other range: the first batch's match may still run
        L = ox.lib()
        assert L.orbx_dev_compute_bow(c.handle, voc, 0, 2 * B, 4) == 0
        c.sync()
        rng = np.random.default_rng(5)
        for s in (0, 15, 16, 31, 32, 47, B, 2 * B - 1):
            kps, desc = c.features(s)
            r = ref_transform(V, desc, 4)
            g = read_bow(c, s, len(kps))
            assert np.array_equal(g["word"], r["word"]) and np.array_equal(g["nid"], r["nid"]), s
            assert g["nf"] == r["nf"] and np.array_equal(g["fn"][:r["nf"]], r["fn"][:r["nf"]]), s
            assert np.array_equal(g["bv"][:r["nw"]].view(np.uint64), r["bv"][:r["nw"]].view(np.uint64)), s
        # Relocalisation of slot 20 against three other frames of the batch
        fk, fd = c.features(20)
        Fv, fa = view(fk, fd, np.zeros(len(fk), np.uint8), ref_transform(V, fd, 4))
        KFs, keep = [], []
        for s in (19, 21, B + 27):
            kk, kd = c.features(s)
            v, a = view(kk, kd, rng.choice(3, len(kk), p=(0.3, 0.6, 0.1)).astype(np.uint8), ref_transform(V, kd, 4))
            KFs.append(v)
            keep.append(a)
        r, outs, nm = search(c, 20, KFs, 0.75, 1)
        assert r == 0
        for i, KF in enumerate(KFs):
            ro, rn = ref_search(0, {"V1": KF, "V2": Fv}, 0.75, 1)
            assert nm[i] == rn and np.array_equal(outs[i][:len(fk)], ro), i
        L.orbx_vocab_destroy(voc)
    finally:
        c.close()


def test_python_wrappers_match_raw_calls(ctx, extracted):
    """Context.compute_bow / read_bow / search_by_bow and Vocabulary give the
    raw C-ABI calls' results."""
    V = make_vocab(k=10, L=5, seed=15)
    voc = ox.Vocabulary(ctx, V["k"], V["L"], V["parent"], V["is_leaf"], V["desc"], V["weight"])
    try:
        assert voc.n_words() == int(V["is_leaf"].sum())
        ctx.compute_bow(voc, 0, 4, 3)
        (bw, bv), (fn, fp, ff), (word, weight, node) = ctx.read_bow(1)
        kps, desc = extracted[1]
        r = ref_transform(V, desc, 3)
        assert np.array_equal(bw, r["bw"][:r["nw"]]) and np.array_equal(bv, r["bv"][:r["nw"]])
        assert np.array_equal(fn, r["fn"][:r["nf"]]) and np.array_equal(fp, r["fp"][:r["nf"] + 1])
        assert np.array_equal(word[:len(kps)], r["word"])
        mp = np.ones(len(kps), np.uint8)
        v, keep = view(kps, desc, mp, r)
        outs, nm = ctx.search_by_bow(0, [v])
        raw = search(ctx, 0, [v], 0.75, 1)
        assert raw[0] == 0 and nm[0] == raw[2][0] and np.array_equal(outs[0], raw[1][0])
    finally:
        voc.close()
