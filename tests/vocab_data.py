"""Synthetic DBoW2 vocabularies (the ORBvoc.txt blob is not in the
reference tree: .MISSING_LARGE_BLOBS:1).  A tree is given the way
TemplatedVocabulary::loadFromTextFile builds it: node 0 the root, then nodes
in file order with their parent id (parents precede children), a leaf flag,
a 32-byte descriptor and a weight.  Children's descriptors are their
parent's with a few bits flipped, so descriptors near a node descend
through it; ~5 % of the words are stopped (weight 0)."""
import ctypes

import numpy as np

from oracle_lib import load, ptr


def make_vocab(k=10, L=4, seed=0, irregular=False):
    rng = np.random.default_rng(seed)
    parent = [0]
    depth = [0]
    desc = [rng.integers(0, 256, 32, dtype=np.uint8)]
    frontier = [0]
    for d in range(1, L + 1):
        nxt = []
        for p in frontier:
            kk = int(rng.integers(1, k + 1)) if irregular else k
            if irregular and d > 1 and rng.random() < 0.15:
                continue                      # this node stays a leaf above depth L
            for _ in range(kk):
                parent.append(p)
                depth.append(d)
                flips = np.packbits((rng.random(256) < 0.25).astype(np.uint8), bitorder="little")
                desc.append(desc[p] ^ flips)
                nxt.append(len(parent) - 1)
        frontier = nxt
    n = len(parent)
    parent = np.array(parent, np.int32)
    has_child = np.zeros(n, bool)
    has_child[parent[1:]] = True
    is_leaf = (~has_child).astype(np.uint8)
    is_leaf[0] = 0
    weight = rng.uniform(0.1, 5.0, n)
    weight[rng.random(n) < 0.05] = 0.0
    return {"k": k, "L": L, "parent": parent, "is_leaf": is_leaf, "desc": np.ascontiguousarray(np.array(desc)),
            "weight": weight}


def features(V, n=1000, seed=1, noise=0.08):
    """Descriptors near random leaves (plus pure noise)."""
    rng = np.random.default_rng(seed)
    leaves = np.nonzero(V["is_leaf"])[0]
    pick = leaves[rng.integers(0, len(leaves), n)]
    d = V["desc"][pick] ^ np.packbits((rng.random((n, 256)) < noise).astype(np.uint8), axis=1, bitorder="little")
    d[: n // 10] = rng.integers(0, 256, (n // 10, 32), dtype=np.uint8)
    return np.ascontiguousarray(d)


def run_ref(V, d, levelsup=4):
    L = load()
    L.orbx_ref_vocab_transform.argtypes = ([ctypes.c_int] * 3 + [ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.c_void_p,
                                                                                   ctypes.c_int] +
                                           [ctypes.c_void_p] * 10)
    n = len(d)
    out = {"word": np.zeros(n, np.int32), "weight": np.zeros(n), "nid": np.zeros(n, np.int32),
           "bw": np.zeros(n, np.uint32), "bv": np.zeros(n), "fn": np.zeros(n, np.uint32),
           "fp": np.zeros(n + 1, np.int32), "ff": np.zeros(n, np.int32)}
    nw, nf = ctypes.c_int(), ctypes.c_int()
    assert L.orbx_ref_vocab_transform(V["k"], V["L"], len(V["parent"]), ptr(V["parent"]), ptr(V["is_leaf"]),
                                      ptr(V["desc"]), ptr(V["weight"]), n, ptr(d), levelsup, ptr(out["word"]),
                                      ptr(out["weight"]), ptr(out["nid"]), ptr(out["bw"]), ptr(out["bv"]),
                                      ctypes.byref(nw), ptr(out["fn"]), ptr(out["fp"]), ptr(out["ff"]),
                                      ctypes.byref(nf)) == 0
    out["nw"], out["nf"] = nw.value, nf.value
    return out
