"""CPU checks of the DBoW2 transform restatement (oracle/ref_vocab.cpp):
the descent against a brute-force numpy walk, BowVector normalisation and
FeatureVector grouping."""
import numpy as np
import pytest

from vocab_data import features, make_vocab, run_ref


def numpy_descend(V, f, levelsup):
    children = {}
    for i in range(1, len(V["parent"])):
        children.setdefault(int(V["parent"][i]), []).append(i)
    node, level, nid = 0, 0, (0 if V["L"] - levelsup <= 0 else -1)
    while node in children:
        level += 1
        ch = children[node]
        dist = [int(np.unpackbits(f ^ V["desc"][c]).sum()) for c in ch]
        node = ch[int(np.argmin(dist))]      # first minimum
        if level == V["L"] - levelsup:
            nid = node
    return node, nid


@pytest.mark.parametrize("irregular,levelsup", [(False, 2), (True, 1), (False, 5)])
def test_transform_matches_numpy_walk(irregular, levelsup):
    V = make_vocab(L=3, seed=2, irregular=irregular)
    d = features(V, n=120, seed=3)
    out = run_ref(V, d, levelsup)
    words = np.cumsum(V["is_leaf"]) - 1
    for i in range(len(d)):
        leaf, nid = numpy_descend(V, d[i], levelsup)
        assert out["word"][i] == words[leaf] and out["nid"][i] == nid
        assert out["weight"][i] == V["weight"][leaf]


def test_bow_and_feature_vectors():
    V = make_vocab(L=4, seed=4)
    d = features(V, n=500, seed=5)
    out = run_ref(V, d, 2)
    keep = out["weight"] > 0
    assert out["nw"] == len(np.unique(out["word"][keep]))
    assert abs(out["bv"][:out["nw"]].sum() - 1.0) < 1e-12
    assert (np.diff(out["bw"][:out["nw"]].astype(np.int64)) > 0).all()
    assert out["fp"][out["nf"]] == keep.sum()
    for j in range(out["nf"]):
        f = out["ff"][out["fp"][j]:out["fp"][j + 1]]
        assert (out["nid"][f] == out["fn"][j]).all() and (np.diff(f) > 0).all()
