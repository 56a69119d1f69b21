"""Independent numpy restatements of ORBmatcher's motion-model and frame-pair
projection searches (B5 SearchByProjection(Frame&, const Frame&, float),
src/ORBmatcher.cc:1507-1620; B7 SearchByProjection(Frame&, Frame&, int,
vector<MapPoint*>&), :519-594; the relocalisation search
SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, float, int),
:1622-1746; the candidates of both Fuse overloads, :1016-1263;
SearchBySim3, :1267-1505; SearchByProjection(KeyFrame*, Scw, ...),
:286-407) with
Frame::GetFeaturesInArea's level range
(src/Frame.cc:199-276), against the oracle's restatement
(oracle/ref_match.cpp) on consecutive bench-sequence frames.

* projection: x3Dc = Rcw x3Dw + tcw in float32 (products summed left to
  right, then + t, as the oracle evaluates the cv::Mat expression -- OpenCV
  2.4's small-matrix gemm order is the one choice shared with the oracle),
  invzc = (float)(1.0 / zc), u = fx xc invzc + cx in float32;
* B5: map points of the last frame that are not outliers; the current
  frame's image bounds; radius th * mvScaleFactors[octave] (the float table
  ORBextractor builds from its double scaleFactor); candidates at octaves
  octave - 1 .. octave + 1 that hold no map point yet (including those taken
  earlier in this call); the first minimum distance, kept at <= TH_HIGH; the
  rotation histogram's three maxima (HISTO_LENGTH 30, bin = round(rot / 30));
* B7: F1's map points, F2's candidates at F1's octave within the window that
  hold no map point; best / second distance, accept at best <= 0.9 second (in
  float) and best <= TH_HIGH; no rotation check.
"""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
from orb_slam_amd import synth
from oracle_lib import RefExtractor, load, ptr
from test_match_numpy import COLS, HISTO, ROWS, Grid, hamming, three_maxima

F32 = np.float32
W, H = 640, 480
CAM = np.array([500.0, 500.0, 320.0, 240.0], np.float32)
TH_HIGH = 100


def scale_factors(nlevels=8, scale=1.2):
    sf = float(F32(scale))        # ORBextractor::scaleFactor is a double holding the float argument
    s = [F32(1.0)]
    for _ in range(1, nlevels):
        s.append(F32(float(s[-1]) * sf))
    return s


def area_levels(g, x, y, r, min_level, max_level):
    """GetFeaturesInArea with its level test (-1 / -1: any level; equal: that level)."""
    x, y, r = F32(x), F32(y), F32(r)
    x0 = max(0, int(np.floor(F32(F32(F32(x - g.minx) - r) * g.winv))))
    if x0 >= COLS:
        return []
    x1 = min(COLS - 1, int(np.ceil(F32(F32(F32(x - g.minx) + r) * g.winv))))
    if x1 < 0:
        return []
    y0 = max(0, int(np.floor(F32(F32(F32(y - g.miny) - r) * g.hinv))))
    if y0 >= ROWS:
        return []
    y1 = min(ROWS - 1, int(np.ceil(F32(F32(F32(y - g.miny) + r) * g.hinv))))
    if y1 < 0:
        return []
    check = not (min_level == -1 and max_level == -1)
    same = check and min_level == max_level
    out = []
    for ix in range(x0, x1 + 1):
        for iy in range(y0, y1 + 1):
            for j in g.cells[ix][iy]:
                k = g.kps[j]
                if check and not same and (k["octave"] < min_level or k["octave"] > max_level):
                    continue
                if same and k["octave"] != min_level:
                    continue
                if abs(F32(k["x"] - x)) > r or abs(F32(k["y"] - y)) > r:
                    continue
                out.append(j)
    return out


def project(T, X):
    T = T.reshape(3, 4)
    xc = [F32(F32(F32(F32(T[r, 0] * X[0]) + F32(T[r, 1] * X[1])) + F32(T[r, 2] * X[2])) + T[r, 3]) for r in range(3)]
    inv = F32(1.0 / float(xc[2]))
    u = F32(F32(F32(CAM[0] * xc[0]) * inv) + CAM[2])
    v = F32(F32(F32(CAM[1] * xc[1]) * inv) + CAM[3])
    return u, v


def rot_bin(a1, a2):
    rot = F32(F32(a1) - F32(a2))
    if rot < 0:
        rot = F32(rot + F32(360.0))
    b = int(np.floor(F32(rot * F32(F32(1.0) / F32(HISTO))) + 0.5))
    return 0 if b == HISTO else b


def motion_search(kc, dc, kl, dl, xyz, valid, assigned, T, th, check_ori):
    g = Grid(kc, W, H)
    sf = scale_factors()
    taken = assigned.astype(bool).copy()
    m = np.full(len(kc), -1, np.int64)
    hist = [[] for _ in range(HISTO)]
    n = 0
    for i in range(len(kl)):
        if not valid[i]:
            continue
        u, v = project(T, xyz[i])
        if u < 0 or u > W or v < 0 or v > H:
            continue
        oct_ = int(kl["octave"][i])
        cand = [c for c in area_levels(g, u, v, F32(F32(th) * sf[oct_]), oct_ - 1, oct_ + 1) if not taken[c]]
        if not cand:
            continue
        dist = hamming(dl[i], dc[np.array(cand)])
        b = int(np.argmin(dist))
        if dist[b] <= TH_HIGH:
            taken[cand[b]] = True
            m[cand[b]] = i
            n += 1
            if check_ori:
                hist[rot_bin(kl["angle"][i], kc["angle"][cand[b]])].append(cand[b])
    if check_ori:
        keep = three_maxima(hist)
        for bi in range(HISTO):
            if bi in keep:
                continue
            for c in hist[bi]:
                m[c] = -1
                n -= 1
    return m, n


def pair_search(k1, d1, k2, d2, xyz, valid, assigned, T, window, nnratio):
    g = Grid(k2, W, H)
    taken = assigned.astype(bool).copy()
    m = np.full(len(k2), -1, np.int64)
    n = 0
    for i in range(len(k1)):
        if not valid[i]:
            continue
        u, v = project(T, xyz[i])
        lvl = int(k1["octave"][i])
        cand = [c for c in area_levels(g, u, v, F32(window), lvl, lvl) if not taken[c]]
        if not cand:
            continue
        dist = hamming(d1[i], d2[np.array(cand)])
        b = int(np.argmin(dist))
        best2 = int(np.sort(dist)[1]) if len(dist) > 1 else 2147483647
        if F32(dist[b]) <= F32(F32(best2) * F32(nnratio)) and dist[b] <= TH_HIGH:
            taken[cand[b]] = True
            m[cand[b]] = i
            n += 1
    return m, n


@pytest.fixture(scope="module")
def feats():
    frames = synth.sequence(W, H, 3, seed=77)
    ex = RefExtractor(1000)
    return [ex(f) for f in frames]


def backproject(k, rng):
    z = rng.uniform(2.0, 6.0, len(k)).astype(np.float32)
    x = (k["x"] - CAM[2]) / CAM[0] * z
    y = (k["y"] - CAM[3]) / CAM[1] * z
    return np.ascontiguousarray(np.stack([x, y, z], 1).astype(np.float32))


def pose(tx=-0.008, ty=-0.004, yaw=0.002):
    c, s = np.cos(yaw), np.sin(yaw)
    return np.array([[c, 0, s, tx], [0, 1, 0, ty], [-s, 0, c, 0.0]], np.float32).reshape(-1).copy()


@pytest.mark.parametrize("th,ori", [(15.0, 1), (7.0, 0), (3.0, 1)])
def test_motion_search_matches_oracle(feats, th, ori):
    (kl, dl), (kc, dc) = feats[1], feats[2]
    rng = np.random.default_rng(int(th))
    xyz = backproject(kl, rng)
    valid = (rng.random(len(kl)) < 0.85).astype(np.uint8)
    assigned = (rng.random(len(kc)) < 0.05).astype(np.uint8)
    T = pose()
    m_np, n_np = motion_search(kc, dc, kl, dl, xyz, valid, assigned, T, th, ori)
    C, Lv = ox.frame_view(kc, dc, W, H), ox.frame_view(kl, dl, W, H)
    mr = np.zeros(len(kc), np.int32)
    nr = ctypes.c_int()
    assert load().orbx_ref_search_by_projection_motion(ctypes.byref(C), ctypes.byref(Lv), ptr(xyz), ptr(valid),
                                                       ptr(assigned), ptr(T), ptr(CAM), th, ori, ptr(mr),
                                                       ctypes.byref(nr)) == 0
    assert n_np == nr.value and n_np > 50
    assert np.array_equal(m_np, mr.astype(np.int64))


@pytest.mark.parametrize("window", [15, 50])
def test_pair_search_matches_oracle(feats, window):
    (k1, d1), (k2, d2) = feats[0], feats[1]
    rng = np.random.default_rng(window)
    xyz = backproject(k1, rng)
    valid = (rng.random(len(k1)) < 0.8).astype(np.uint8)
    assigned = (rng.random(len(k2)) < 0.1).astype(np.uint8)
    T = pose()
    m_np, n_np = pair_search(k1, d1, k2, d2, xyz, valid, assigned, T, window, 0.9)
    F1, F2 = ox.frame_view(k1, d1, W, H), ox.frame_view(k2, d2, W, H)
    mr = np.zeros(len(k2), np.int32)
    nr = ctypes.c_int()
    assert load().orbx_ref_search_by_projection_pair(ctypes.byref(F1), ctypes.byref(F2), ptr(xyz), ptr(valid),
                                                     ptr(assigned), ptr(T), ptr(CAM), window, 0.9, ptr(mr),
                                                     ctypes.byref(nr)) == 0
    assert n_np == nr.value and n_np > 50
    assert np.array_equal(m_np, mr.astype(np.int64))


def test_scale_factors_match_extractor():
    e = RefExtractor(1000)
    s, inv = np.zeros(8, np.float32), np.zeros(8, np.float32)
    assert e.L.orbx_ref_scale_factors(e.h, ptr(s), ptr(inv), 8) == 8
    assert np.array_equal(np.array(scale_factors(), np.float32), s)


def frame_kf_search(kf, kf_desc, fk, fd, pos, dmin, valid, assigned, T, th, orb_dist, check_ori):
    """SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, float, int)
    (src/ORBmatcher.cc:1622-1746): the KF's map points (valid = not bad and
    not already found) projected into the frame; predicted level from
    |X - Ow| / GetMinDistanceInvariance() by lower_bound over the float scale
    table; radius th * scale; the frame's keypoints at levels pred - 1 ..
    pred + 1 without a map point; first minimum <= ORBdist; rotation check
    with the KF keypoint's angle.  Ow = -Rcw^T tcw in float (left to right,
    the oracle's evaluation of the cv::Mat expression); cv::norm accumulates
    the squares in double."""
    g = Grid(fk, W, H)
    sf = scale_factors()
    Tm = T.reshape(4, 4)[:3] if T.size == 16 else T.reshape(3, 4)
    R, t = Tm[:, :3], Tm[:, 3]
    Ow = [F32(-F32(F32(F32(R[0, c] * t[0]) + F32(R[1, c] * t[1])) + F32(R[2, c] * t[2]))) for c in range(3)]
    taken = assigned.astype(bool).copy()
    m = np.full(len(fk), -1, np.int64)
    hist = [[] for _ in range(HISTO)]
    n = 0
    for i in range(len(kf)):
        if not valid[i]:
            continue
        X = pos[i]
        u, v = project(np.concatenate([Tm[r] for r in range(3)]).astype(np.float32), X)
        if u < 0 or u > W or v < 0 or v > H:
            continue
        PO = [F32(X[c] - Ow[c]) for c in range(3)]
        dist3 = F32(np.sqrt(sum(float(p) * float(p) for p in PO)))
        ratio = F32(dist3 / F32(dmin[i]))
        pred = min(int(np.searchsorted(np.array(sf, np.float32), ratio, side="left")), len(sf) - 1)
        cand = [c for c in area_levels(g, u, v, F32(F32(th) * sf[pred]), pred - 1, pred + 1) if not taken[c]]
        if not cand:
            continue
        dist = hamming(kf_desc[i], fd[np.array(cand)])
        b = int(np.argmin(dist))
        if dist[b] <= orb_dist:
            taken[cand[b]] = True
            m[cand[b]] = i
            n += 1
            if check_ori:
                hist[rot_bin(kf["angle"][i], fk["angle"][cand[b]])].append(cand[b])
    if check_ori:
        keep = three_maxima(hist)
        for bi in range(HISTO):
            if bi in keep:
                continue
            for c in hist[bi]:
                m[c] = -1
                n -= 1
    return m, n


@pytest.mark.parametrize("seed,th,orb_dist,ori", [(1, 10.0, 100, 1), (2, 5.0, 64, 0)])
def test_frame_kf_search_matches_oracle(seed, th, orb_dist, ori):
    import proj_data as pd
    from test_proj_oracle import ref_proj_frame_kf, seq_case
    k1, d1, k2, d2, T2, mps, rng = seq_case(seed)
    valid = (rng.random(len(k1)) < 0.8).astype(np.uint8)
    assigned = (rng.random(len(k2)) < 0.1).astype(np.uint8)
    a = mps[1]
    got, n = frame_kf_search(k1, a["desc"], k2, d2, a["pos"], a["min_dist"], valid, assigned,
                             np.ascontiguousarray(T2, np.float32), th, orb_dist, ori)
    want, nw = ref_proj_frame_kf(pd.view(k2, d2), pd.view(k1, d1), mps, valid, assigned, T2, th, orb_dist, ori)
    assert n == nw and n > 100
    assert np.array_equal(got, want.astype(np.int64))


def fuse_candidates(k, d, pos, normal, dmin, dmax, mdesc, T, sim3, th):
    """The state-free part of ORBmatcher::Fuse (KF, vpMapPoints) (src/
    ORBmatcher.cc:1016-1134) and Fuse (KF, Scw, vpPoints) (:1136-1263) per
    map point: camera frame (Scw decomposed as scw = sqrt(row0 . row0) in
    double, Rcw = sRcw / scw and tcw / scw through a double reciprocal),
    positive depth, 1/z in float (KF overload) or 1.0/z in double (Scw
    overload), KeyFrame::IsInImage (half-open), the scale-invariance distance
    range, the 60-degree viewing test PO . Pn >= 0.5 |PO| in double, the
    predicted level, and the first minimum over the keypoints in the radius
    whose octave lies in [pred - 1, pred]."""
    g = Grid(k, W, H)
    sf = scale_factors()
    T = T.reshape(4, 4)
    if sim3:
        scw = F32(np.sqrt(sum(float(T[0, c]) * float(T[0, c]) for c in range(3))))
        inv = 1.0 / float(scw)
        R = np.array([[F32(float(T[r, c]) * inv) for c in range(3)] for r in range(3)], np.float32)
        t = np.array([F32(float(T[r, 3]) * inv) for r in range(3)], np.float32)
    else:
        R, t = T[:3, :3], T[:3, 3]
    Ow = [F32(-F32(F32(F32(R[0, c] * t[0]) + F32(R[1, c] * t[1])) + F32(R[2, c] * t[2]))) for c in range(3)]
    n = len(pos)
    bi = np.full(n, -1, np.int64)
    bd = np.full(n, 2147483647, np.int64)
    for m in range(n):
        X = pos[m]
        pc = [F32(F32(F32(F32(R[r, 0] * X[0]) + F32(R[r, 1] * X[1])) + F32(R[r, 2] * X[2])) + t[r]) for r in range(3)]
        if pc[2] < 0:
            continue
        invz = F32(1.0 / float(pc[2])) if sim3 else F32(F32(1.0) / pc[2])
        u = F32(F32(CAM[0] * F32(pc[0] * invz)) + CAM[2])
        v = F32(F32(CAM[1] * F32(pc[1] * invz)) + CAM[3])
        if not (0 <= u < W and 0 <= v < H):
            continue
        PO = [F32(X[c] - Ow[c]) for c in range(3)]
        dist3 = F32(np.sqrt(sum(float(p) * float(p) for p in PO)))
        if dist3 < dmin[m] or dist3 > dmax[m]:
            continue
        if sum(float(PO[c]) * float(normal[m, c]) for c in range(3)) < 0.5 * float(dist3):
            continue
        pred = min(int(np.searchsorted(np.array(sf, np.float32), F32(dist3 / F32(dmin[m])), side="left")), len(sf) - 1)
        cand = [c for c in area_levels(g, u, v, F32(F32(th) * sf[pred]), -1, -1)
                if pred - 1 <= k["octave"][c] <= pred]
        if not cand:
            continue
        dist = hamming(mdesc[m], d[np.array(cand)])
        b = int(np.argmin(dist))
        bi[m], bd[m] = cand[b], int(dist[b])
    return bi, bd


@pytest.mark.parametrize("sim3,scale,th", [(0, 1.0, 3.0), (1, 1.5, 3.0), (1, 0.7, 6.0)])
def test_fuse_candidates_match_oracle(sim3, scale, th):
    from test_proj_oracle import ref_fuse, seq_case
    import proj_data as pd
    k1, d1, k2, d2, T2, mps, rng = seq_case(3)
    S = np.ascontiguousarray(T2, np.float32).copy()
    if sim3:
        S[:3, :] *= np.float32(scale)
    a = mps[1]
    got_i, got_d = fuse_candidates(k2, d2, a["pos"], a["normal"], a["min_dist"], a["max_dist"], a["desc"], S, sim3, th)
    want_i, want_d = ref_fuse(pd.view(k2, d2), mps, S, sim3, th)
    assert np.count_nonzero(want_i >= 0) > 100
    assert np.array_equal(got_i, want_i.astype(np.int64))
    assert np.array_equal(got_d[got_i >= 0], want_d[want_i >= 0].astype(np.int64))


def search_by_sim3(k1, d1, k2, d2, m1, v1, m2, v2, T1, T2, s12, R12, t12, prior, th):
    """ORBmatcher::SearchBySim3 (src/ORBmatcher.cc:1267-1505): KF1's map
    points through R1w, t1w then sR21 = (1.0 / s12) R12^T (double scale),
    t21 = -sR21 t12 into KF2, and KF2's through R2w, t2w then sR12 = s12 R12
    into KF1; positive depth, 1.0/z in double, IsInImage, the distance range
    on |p3Dc| (no viewing test), predicted level, best keypoint in the radius
    at octaves [pred - 1, pred] with distance <= TH_HIGH; kept when the two
    directions agree.  prior: -2 no match yet, -1 a match whose point is not
    in KF2, >= 0 its KF2 index (vbAlreadyMatched1 / 2)."""
    sf = scale_factors()
    R12 = R12.reshape(3, 3)
    sR12 = np.array([[F32(float(s12) * float(R12[r, c])) for c in range(3)] for r in range(3)], np.float32)
    inv = 1.0 / float(s12)
    sR21 = np.array([[F32(inv * float(R12[c, r])) for c in range(3)] for r in range(3)], np.float32)
    t21 = np.array([F32(-F32(F32(F32(sR21[r, 0] * t12[0]) + F32(sR21[r, 1] * t12[1])) + F32(sR21[r, 2] * t12[2])))
                    for r in range(3)], np.float32)
    already1 = prior != -2
    already2 = np.zeros(len(k2), bool)
    for i in range(len(k1)):
        if prior[i] >= 0:
            already2[prior[i]] = True

    def xf(R, t, X):
        return [F32(F32(F32(F32(R[r, 0] * X[0]) + F32(R[r, 1] * X[1])) + F32(R[r, 2] * X[2])) + t[r]) for r in range(3)]

    grids = {id(k1): Grid(k1, W, H), id(k2): Grid(k2, W, H)}

    def one(kd, dd, mp, i, Rw, tw, sR, tt):
        pc = xf(sR, tt, np.array(xf(Rw, tw, mp["pos"][i]), np.float32))
        if pc[2] < 0:
            return -1
        invz = F32(1.0 / float(pc[2]))
        u = F32(F32(CAM[0] * F32(pc[0] * invz)) + CAM[2])
        v = F32(F32(CAM[1] * F32(pc[1] * invz)) + CAM[3])
        if not (0 <= u < W and 0 <= v < H):
            return -1
        dist3 = F32(np.sqrt(sum(float(p) * float(p) for p in pc)))
        if dist3 < mp["min_dist"][i] or dist3 > mp["max_dist"][i]:
            return -1
        pred = min(int(np.searchsorted(np.array(sf, np.float32), F32(dist3 / F32(mp["min_dist"][i])), side="left")),
                   len(sf) - 1)
        cand = [c for c in area_levels(grids[id(kd)], u, v, F32(F32(th) * sf[pred]), -1, -1)
                if pred - 1 <= kd["octave"][c] <= pred]
        if not cand:
            return -1
        dist = hamming(mp["desc"][i], dd[np.array(cand)])
        b = int(np.argmin(dist))
        return cand[b] if dist[b] <= TH_HIGH else -1

    T1, T2 = T1.reshape(4, 4), T2.reshape(4, 4)
    match1 = [one(k2, d2, m1, i, T1[:3, :3], T1[:3, 3], sR21, t21) if v1[i] and not already1[i] else -1
              for i in range(len(k1))]
    match2 = [one(k1, d1, m2, i, T2[:3, :3], T2[:3, 3], sR12, t12) if v2[i] and not already2[i] else -1
              for i in range(len(k2))]
    new = np.full(len(k1), -1, np.int64)
    for i1, i2 in enumerate(match1):
        if i2 >= 0 and match2[i2] == i1:
            new[i1] = i2
    return new, int((new >= 0).sum())


@pytest.mark.parametrize("seed,prior_frac,th", [(0, 0.1, 7.5), (2, 0.3, 4.0)])
def test_search_by_sim3_matches_oracle(seed, prior_frac, th):
    from test_proj_oracle import ref_sim3, sim3_case
    K1, K2, m1, v1, m2, v2, T1, T2, s12, R12, t12, prior, (k1, d1, k2, d2) = sim3_case(seed, prior_frac)
    got, n = search_by_sim3(k1, d1, k2, d2, m1[1], v1, m2[1], v2, T1, T2, s12, R12, t12, prior, th)
    want, nw = ref_sim3(K1, K2, m1, v1, m2, v2, T1, T2, s12, R12, t12, prior, th)
    assert n == nw and n > 100
    assert np.array_equal(got, want.astype(np.int64))


def kf_scw_search(k, d, mp, skip, Scw, th, matched):
    """SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th) (src/
    ORBmatcher.cc:286-407): Fuse (KF, Scw)'s geometry with 1/z in float,
    radius th * scale, candidates in the radius at octaves [pred - 1, pred]
    whose vpMatched entry is empty (including entries set earlier in this
    call), first minimum <= TH_LOW assigned."""
    g = Grid(k, W, H)
    sf = scale_factors()
    T = Scw.reshape(4, 4)
    scw = F32(np.sqrt(sum(float(T[0, c]) * float(T[0, c]) for c in range(3))))
    inv = 1.0 / float(scw)
    R = np.array([[F32(float(T[r, c]) * inv) for c in range(3)] for r in range(3)], np.float32)
    t = np.array([F32(float(T[r, 3]) * inv) for r in range(3)], np.float32)
    Ow = [F32(-F32(F32(F32(R[0, c] * t[0]) + F32(R[1, c] * t[1])) + F32(R[2, c] * t[2]))) for c in range(3)]
    out = matched.astype(np.int64).copy()
    n = 0
    for m in range(len(mp["pos"])):
        if skip[m]:
            continue
        X = mp["pos"][m]
        pc = [F32(F32(F32(F32(R[r, 0] * X[0]) + F32(R[r, 1] * X[1])) + F32(R[r, 2] * X[2])) + t[r]) for r in range(3)]
        if pc[2] < 0:
            continue
        invz = F32(F32(1.0) / pc[2])
        u = F32(F32(CAM[0] * F32(pc[0] * invz)) + CAM[2])
        v = F32(F32(CAM[1] * F32(pc[1] * invz)) + CAM[3])
        if not (0 <= u < W and 0 <= v < H):
            continue
        PO = [F32(X[c] - Ow[c]) for c in range(3)]
        dist3 = F32(np.sqrt(sum(float(p) * float(p) for p in PO)))
        if dist3 < mp["min_dist"][m] or dist3 > mp["max_dist"][m]:
            continue
        if sum(float(PO[c]) * float(mp["normal"][m, c]) for c in range(3)) < 0.5 * float(dist3):
            continue
        pred = min(int(np.searchsorted(np.array(sf, np.float32), F32(dist3 / F32(mp["min_dist"][m])), side="left")),
                   len(sf) - 1)
        cand = [c for c in area_levels(g, u, v, F32(F32(th) * sf[pred]), -1, -1)
                if out[c] < 0 and pred - 1 <= k["octave"][c] <= pred]
        if not cand:
            continue
        dist = hamming(mp["desc"][m], d[np.array(cand)])
        b = int(np.argmin(dist))
        if dist[b] <= 50:
            out[cand[b]] = m
            n += 1
    return out, n


@pytest.mark.parametrize("seed,scale,th", [(0, 1.5, 10), (4, 0.8, 5)])
def test_kf_scw_search_matches_oracle(seed, scale, th):
    import proj_data as pd
    from test_proj_oracle import ref_proj_kf_sim3, seq_case
    k1, d1, k2, d2, T2, mps, rng = seq_case(seed)
    S = np.ascontiguousarray(T2, np.float32).copy()
    S[:3, :] *= np.float32(scale)
    skip = (rng.random(len(k1)) < 0.1).astype(np.uint8)
    matched = np.full(len(k2), -1, np.int32)
    matched[rng.random(len(k2)) < 0.05] = 10 ** 6
    got, n = kf_scw_search(k2, d2, mps[1], skip, S, th, matched)
    want, nw = ref_proj_kf_sim3(pd.view(k2, d2), mps, skip, S, th, matched)
    assert n == nw and n > 100
    assert np.array_equal(got, want.astype(np.int64))
