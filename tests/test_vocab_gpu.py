"""GPU DBoW2 vocabulary-tree descent (TemplatedVocabulary::transform,
Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1259) through the C ABI
against the CPU restatement: per-feature word / weight / node, BowVector and
FeatureVector identical (values bit-identical)."""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
from vocab_data import features, make_vocab, run_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
    yield c
    c.close()


def gpu_transform(ctx, V, d, levelsup):
    L = ox.lib()
    voc = ctypes.c_void_p()
    assert L.orbx_vocab_create(ctx.handle, V["k"], V["L"], len(V["parent"]), ox._ptr(V["parent"]),
                               ox._ptr(V["is_leaf"]), ox._ptr(V["desc"]), ox._ptr(V["weight"]),
                               ctypes.byref(voc)) == 0
    try:
        assert L.orbx_vocab_n_words(voc) == int(V["is_leaf"].sum())
        n = len(d)
        out = {"word": np.zeros(n, np.int32), "weight": np.zeros(n), "nid": np.zeros(n, np.int32),
               "bw": np.zeros(n, np.uint32), "bv": np.zeros(n), "fn": np.zeros(n, np.uint32),
               "fp": np.zeros(n + 1, np.int32), "ff": np.zeros(n, np.int32)}
        nw, nf = ctypes.c_int(), ctypes.c_int()
        assert L.orbx_vocab_transform(ctx.handle, voc, n, ox._ptr(d), levelsup, ox._ptr(out["word"]),
                                      ox._ptr(out["weight"]), ox._ptr(out["nid"]), ox._ptr(out["bw"]),
                                      ox._ptr(out["bv"]), ctypes.byref(nw), ox._ptr(out["fn"]), ox._ptr(out["fp"]),
                                      ox._ptr(out["ff"]), ctypes.byref(nf)) == 0
        out["nw"], out["nf"] = nw.value, nf.value
        return out
    finally:
        L.orbx_vocab_destroy(voc)


@pytest.mark.parametrize("k,L,irregular,levelsup,n", [(10, 4, False, 4, 1000), (10, 6, False, 4, 2000),
                                                      (6, 5, True, 2, 1500), (10, 3, False, 6, 300)])
def test_vocab_transform_matches_oracle(ctx, k, L, irregular, levelsup, n):
    V = make_vocab(k=k, L=L, seed=k + L, irregular=irregular)
    d = features(V, n=n, seed=L)
    r = run_ref(V, d, levelsup)
    g = gpu_transform(ctx, V, d, levelsup)
    for key in ["word", "weight", "nid"]:
        assert np.array_equal(g[key], r[key]), key
    assert g["nw"] == r["nw"] and g["nf"] == r["nf"]
    assert np.array_equal(g["bw"][:r["nw"]], r["bw"][:r["nw"]])
    assert np.array_equal(g["bv"][:r["nw"]], r["bv"][:r["nw"]])
    assert np.array_equal(g["fn"][:r["nf"]], r["fn"][:r["nf"]])
    assert np.array_equal(g["fp"][:r["nf"] + 1], r["fp"][:r["nf"] + 1])
    assert np.array_equal(g["ff"], r["ff"])
