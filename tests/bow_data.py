"""Synthetic keyframe pairs for the vocabulary-node searches
(SearchByBoW / SearchForTriangulation, src/ORBmatcher.cc:155-283, 715-1014).

Two cameras (KF1 at the origin, KF2 moved by `baseline` and rotated) see a
cloud of 3D points.  A fraction of KF1's features has a true correspondence
in KF2 (projection + noise, descriptor with a few flipped bits, orientation
shifted by a common rotation plus noise) that usually falls in the same
vocabulary node; the rest are unrelated.  Node ids, map-point states and
octaves are random, so every branch of the three searches is exercised.
F12 = K^-T [t12]x R12 K^-1 (Tracking/LocalMapping's ComputeF12), float.

Returns orbx_bow_view structs over arrays kept alive by the returned dict.
"""
import ctypes

import numpy as np

import orb_slam_amd as ox

K = np.array([[500.0, 0, 320.0], [0, 500.0, 240.0], [0, 0, 1]])


class BowView(ctypes.Structure):
    _fields_ = [("keys", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("n", ctypes.c_int), ("mp", ctypes.c_void_p),
                ("n_nodes", ctypes.c_int), ("node_id", ctypes.c_void_p), ("node_ptr", ctypes.c_void_p),
                ("feat_idx", ctypes.c_void_p)]


def _rot(w):
    th = np.linalg.norm(w)
    Kx = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th < 1e-12:
        return np.eye(3)
    return np.eye(3) + np.sin(th) / th * Kx + (1 - np.cos(th)) / th ** 2 * Kx @ Kx


def feature_vector(node_of):
    """CSR FeatureVector: node ids ascending, features ascending per node."""
    order = np.lexsort((np.arange(len(node_of)), node_of))
    ids, starts = np.unique(node_of[order], return_index=True)
    ptr = np.append(starts, len(order)).astype(np.int32)
    return ids.astype(np.uint32), ptr, order.astype(np.int32)


def make_view(kps, desc, mp, node_of):
    ids, ptr, feat = feature_vector(node_of)
    arrs = {"kps": np.ascontiguousarray(kps), "desc": np.ascontiguousarray(desc, np.uint8),
            "mp": np.ascontiguousarray(mp, np.uint8), "ids": ids, "ptr": ptr, "feat": feat}
    v = BowView()
    v.keys = arrs["kps"].ctypes.data
    v.desc = arrs["desc"].ctypes.data
    v.n = len(kps)
    v.mp = arrs["mp"].ctypes.data
    v.n_nodes = len(ids)
    v.node_id = ids.ctypes.data if len(ids) else None
    v.node_ptr = ptr.ctypes.data
    v.feat_idx = feat.ctypes.data if len(feat) else None
    return v, arrs


def make_pair(n1=1000, n2=1000, n_nodes=80, match_frac=0.6, same_node=0.9, seed=0, mp_probs=(0.4, 0.5, 0.1),
              baseline=0.3, node_pool=None):
    rng = np.random.default_rng(seed)
    R2 = _rot(rng.normal(0, 0.05, 3))
    t2 = np.array([-baseline, 0.02, 0.01])
    # KF1 features: projections of points 2-8 m in front
    u1 = rng.uniform(0, 640, n1)
    v1 = rng.uniform(0, 480, n1)
    z = rng.uniform(2.0, 8.0, n1)
    X = np.stack([(u1 - 320) / 500 * z, (v1 - 240) / 500 * z, z], 1)
    Xc2 = X @ R2.T + t2
    uv2 = Xc2[:, :2] / Xc2[:, 2:] * 500 + np.array([320.0, 240.0])
    pool = node_pool if node_pool is not None else np.sort(rng.choice(100000, n_nodes, replace=False))
    node1 = pool[rng.integers(0, len(pool), n1)]
    desc1 = rng.integers(0, 256, (n1, 32), dtype=np.uint8)
    ang1 = rng.uniform(0, 360, n1).astype(np.float32)
    oct1 = rng.integers(0, 8, n1)
    # KF2: first the correspondences of a random subset, then unrelated features
    nm = min(int(match_frac * n1), n2)
    src = rng.choice(n1, nm, replace=False)
    kp2 = np.zeros((n2, 2))
    kp2[:nm] = uv2[src] + rng.normal(0, 0.7, (nm, 2))
    kp2[nm:] = np.stack([rng.uniform(0, 640, n2 - nm), rng.uniform(0, 480, n2 - nm)], 1)
    desc2 = rng.integers(0, 256, (n2, 32), dtype=np.uint8)
    flips = (rng.random((nm, 256)) < rng.uniform(0.01, 0.2, (nm, 1))).astype(np.uint8)
    desc2[:nm] = desc1[src] ^ np.packbits(flips, axis=1, bitorder="little")
    node2 = pool[rng.integers(0, len(pool), n2)]
    keep = rng.random(nm) < same_node
    node2[:nm][keep] = node1[src][keep]
    ang2 = rng.uniform(0, 360, n2).astype(np.float32)
    ang2[:nm] = np.mod(ang1[src] - 20.0 + rng.normal(0, 4, nm), 360).astype(np.float32)
    oct2 = rng.integers(0, 8, n2)
    oct2[:nm] = oct1[src]
    perm = rng.permutation(n2)   # correspondences not in index order

    def keys(xy, ang, octv):
        k = np.zeros(len(xy), ox.KEYPOINT)
        k["x"], k["y"] = xy[:, 0], xy[:, 1]
        k["size"] = 31.0
        k["angle"] = ang
        k["response"] = 10.0
        k["octave"] = octv
        k["class_id"] = -1
        return k

    k1 = keys(np.stack([u1, v1], 1), ang1, oct1)
    k2 = keys(kp2[perm], ang2[perm], oct2[perm])
    mp1 = rng.choice(3, n1, p=mp_probs).astype(np.uint8)
    mp2 = rng.choice(3, n2, p=mp_probs).astype(np.uint8)
    V1, a1 = make_view(k1, desc1, mp1, node1)
    V2, a2 = make_view(k2, desc2[perm], mp2, node2[perm])
    # F12 = K^-T [t12]x R12 K^-1 with R12 = R1w R2w^T, t12 = -R12 t2w (KF1 at the origin)
    R12 = R2.T
    t12 = -R12 @ t2
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
    Ki = np.linalg.inv(K)
    F12 = (Ki.T @ tx @ R12 @ Ki).astype(np.float32).reshape(-1).copy()
    s = np.float32(1.0)
    sig2 = []
    for _ in range(8):
        sig2.append(np.float32(s * s))
        s = np.float32(s * np.float32(1.2))
    return {"V1": V1, "V2": V2, "keep": (a1, a2), "F12": F12, "sigma2": np.array(sig2, np.float32)}
