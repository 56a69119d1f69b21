"""Synthetic local maps for Tracking::SearchReferencePointsInFrustum
(src/Tracking.cc:701-752): the ctypes view of orbx_local_map_query and a
generator of local map points around a frame's keypoints (test data only)."""
import ctypes

import numpy as np

import orb_slam_amd as ox

CAM = np.array([500.0, 500.0, 320.0, 240.0], np.float32)
vp = ctypes.c_void_p


class LocalMapQuery(ctypes.Structure):
    _fields_ = [("frame", vp), ("Rcw", vp), ("tcw", vp), ("Ow", vp), ("cam", vp), ("n_mp", ctypes.c_int),
                ("mp_pos", vp), ("mp_normal", vp), ("mp_dist", vp), ("mp_skip", vp), ("mp_desc", vp),
                ("f_assigned", vp), ("view_cos_limit", ctypes.c_float), ("th", ctypes.c_float),
                ("nnratio", ctypes.c_float), ("in_view", vp), ("proj_xy", vp), ("pred_level", vp),
                ("view_cos", vp), ("matches_f", vp), ("n_in_view", ctypes.c_int), ("n_matches", ctypes.c_int)]


def pose(tx=-0.008, ty=-0.004, yaw=0.002):
    c, s = np.cos(yaw), np.sin(yaw)
    R = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]], np.float32)
    t = np.array([tx, ty, 0.0], np.float32)
    Ow = (-(R.T.astype(np.float64) @ t.astype(np.float64))).astype(np.float32)
    return np.ascontiguousarray(R.reshape(-1)), t, Ow


def make_case(km, dm, kf, df, w, h, seed, nlevels=8, scale=1.2, extra=300, th=1.0):
    """Local map points: the map frame's keypoints back-projected from the
    identity pose (with their descriptors, noisy normals and the distance
    range ORB-SLAM derives from the observing level,
    MapPoint::UpdateNormalAndDepth), plus `extra` random points of which
    some lie behind the camera, outside the image, outside their distance
    range or at a grazing viewing angle.  Returns the numpy arrays that keep
    a LocalMapQuery alive and the query itself."""
    r = np.random.default_rng(seed)
    n0 = len(km)
    z = r.uniform(2.0, 6.0, n0)
    P0 = np.stack([(km["x"] - CAM[2]) / CAM[0] * z, (km["y"] - CAM[3]) / CAM[1] * z, z], 1)
    P1 = np.stack([r.uniform(-8, 8, extra), r.uniform(-6, 6, extra), r.uniform(-3, 9, extra)], 1)
    P = np.concatenate([P0, P1]).astype(np.float32)
    n = len(P)
    dist = np.linalg.norm(P.astype(np.float64), axis=1)
    normal = P / np.maximum(dist[:, None], 1e-9)
    normal = normal + r.normal(0, 0.3, normal.shape) * (r.random((n, 1)) < 0.2)   # some grazing views
    normal = (normal / np.linalg.norm(normal, axis=1, keepdims=True)).astype(np.float32)
    level = np.concatenate([km["octave"], r.integers(0, nlevels, extra)]).astype(np.int64)
    sf = scale ** np.arange(nlevels)
    dmax = dist * sf[level] * r.uniform(0.7, 1.3, n)
    dmin = dmax / sf[-1]
    mp_dist = np.ascontiguousarray(np.stack([dmin, dmax], 1).astype(np.float32))
    desc = np.concatenate([dm, r.integers(0, 256, (extra, 32), dtype=np.uint8)])
    skip = (r.random(n) < 0.05).astype(np.uint8)
    assigned = (r.random(len(kf)) < 0.05).astype(np.uint8)
    Rcw, tcw, Ow = pose(yaw=float(r.uniform(-0.004, 0.004)))
    F = ox.frame_view(kf, df, w, h, nlevels, scale)
    arrs = dict(F=F, kf=kf, df=df, Rcw=Rcw, tcw=tcw, Ow=Ow, cam=CAM.copy(), pos=np.ascontiguousarray(P),
                normal=np.ascontiguousarray(normal), dist=mp_dist, skip=skip, desc=np.ascontiguousarray(desc),
                assigned=assigned, in_view=np.zeros(n, np.uint8), proj=np.zeros((n, 2), np.float32),
                pred=np.zeros(n, np.int32), cos=np.zeros(n, np.float32), matches=np.zeros(len(kf), np.int32))
    q = LocalMapQuery()
    q.frame = ctypes.addressof(F)
    for field, key in (("Rcw", "Rcw"), ("tcw", "tcw"), ("Ow", "Ow"), ("cam", "cam"), ("mp_pos", "pos"),
                       ("mp_normal", "normal"), ("mp_dist", "dist"), ("mp_skip", "skip"), ("mp_desc", "desc"),
                       ("f_assigned", "assigned"), ("in_view", "in_view"), ("proj_xy", "proj"),
                       ("pred_level", "pred"), ("view_cos", "cos"), ("matches_f", "matches")):
        setattr(q, field, arrs[key].ctypes.data)
    q.n_mp = n
    q.view_cos_limit = 0.5
    q.th = th
    q.nnratio = 0.8
    return arrs, q


def outputs(arrs, q):
    return (arrs["in_view"].copy(), arrs["proj"].copy(), arrs["pred"].copy(), arrs["cos"].copy(),
            arrs["matches"].copy(), q.n_in_view, q.n_matches)
