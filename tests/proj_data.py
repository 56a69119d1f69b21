"""Synthetic keyframes and map points for the keyframe projection searches
(Fuse, SearchBySim3; src/ORBmatcher.cc:1016-1505) and for
ComputeDistinctiveDescriptors (src/MapPoint.cc:185-250).

Keyframes are ORB features (oracle extractor) of two frames of a synthetic
sequence; frame 1 is frame 0 shifted by a few pixels, which a camera
translation reproduces for points at a common depth.  Map points are the
keyframes' keypoints back-projected (depth z0, a fraction jittered) with the
MapPoint::UpdateNormalAndDepth distance range and the keypoint's descriptor.
"""
import ctypes

import numpy as np

import orb_slam_amd as ox
from orb_slam_amd import synth
from oracle_lib import RefExtractor

W, H = 640, 480
CAM = np.array([500.0, 500.0, 320.0, 240.0], np.float32)
Z0 = 4.0
_cache = {}


class MapPointView(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("pos", ctypes.c_void_p), ("normal", ctypes.c_void_p),
                ("min_dist", ctypes.c_void_p), ("max_dist", ctypes.c_void_p), ("desc", ctypes.c_void_p)]


def keyframes():
    if "kf" not in _cache:
        frames = synth.sequence(W, H, 2, seed=31)
        ex = RefExtractor(1000)
        feats = [ex(f) for f in frames]
        (k1, d1), (k2, d2) = feats
        # image shift between the frames from brute-force matches
        D = np.unpackbits(d1[:, None, :] ^ d2[None, :, :], axis=2).sum(2)
        j = D.argmin(1)
        good = D[np.arange(len(k1)), j] < 20
        du = float(np.median(k2["x"][j[good]] - k1["x"][good]))
        dv = float(np.median(k2["y"][j[good]] - k1["y"][good]))
        _cache["kf"] = (k1, d1, k2, d2, du, dv)
    return _cache["kf"]


def view(k, d):
    return ox.frame_view(k, d, W, H)


def pose_T(t):
    T = np.eye(4, dtype=np.float32)
    T[:3, 3] = t
    return T


def mappoints(k, d, T, rng, jitter=0.3, flip=0.05):
    """World points of keypoints k seen from camera pose T (Tcw, pure
    translation), plus the MapPoint fields the searches read."""
    n = len(k)
    z = np.full(n, Z0)
    j = rng.random(n) < jitter
    z[j] *= rng.uniform(0.7, 1.4, j.sum())
    Xc = np.stack([(k["x"] - CAM[2]) / CAM[0] * z, (k["y"] - CAM[3]) / CAM[1] * z, z], 1)
    Xw = (Xc - T[:3, 3]).astype(np.float32)
    Ow = -T[:3, 3]
    PO = Xw - Ow
    dist = np.linalg.norm(PO, axis=1).astype(np.float32)
    nrm = (PO / dist[:, None] + rng.normal(0, 0.05, (n, 3))).astype(np.float32)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    scale = np.float32(1.2) ** np.arange(8, dtype=np.float32)
    lvl = k["octave"]
    # MapPoint::UpdateNormalAndDepth's range (src/MapPoint.cc:308-309), the
    # lower bound widened by 5 % so the predicted level brackets the octave
    dmin = (np.float32(1.05) / np.float32(1.2) * dist / scale[lvl]).astype(np.float32)
    dmax = (np.float32(1.2) * dist * scale[7 - lvl]).astype(np.float32)
    bits = (rng.random((n, 256)) < flip).astype(np.uint8)
    desc = d ^ np.packbits(bits, axis=1, bitorder="little")
    arrs = {"pos": np.ascontiguousarray(Xw), "normal": np.ascontiguousarray(nrm.astype(np.float32)),
            "min_dist": dmin, "max_dist": dmax, "desc": np.ascontiguousarray(desc)}
    v = MapPointView()
    v.n = n
    for key, a in arrs.items():
        setattr(v, key, a.ctypes.data)
    return v, arrs


def distinctive_sets(n_mp=400, seed=0, sizes=None):
    rng = np.random.default_rng(seed)
    if sizes is None:
        sizes = rng.integers(0, 30, n_mp)
        sizes[:4] = [0, 1, 2, 3]
        sizes[4:8] = [64, 65, 130, 257]
    ptr = np.zeros(len(sizes) + 1, np.int32)
    ptr[1:] = np.cumsum(sizes)
    desc = np.zeros((int(ptr[-1]), 32), np.uint8)
    for m, s in enumerate(sizes):
        base = rng.integers(0, 256, 32, dtype=np.uint8)
        for i in range(s):
            rate = 0.5 if rng.random() < 0.2 else rng.uniform(0.0, 0.15)
            desc[ptr[m] + i] = base ^ np.packbits((rng.random(256) < rate).astype(np.uint8), bitorder="little")
    return ptr, desc
