"""Frame::isInFrustum (src/Frame.cc:136-197) + the local-map
SearchByProjection (src/ORBmatcher.cc:49-125) as Tracking::
SearchReferencePointsInFrustum runs them (src/Tracking.cc:701-752), on the
device with no host pass over the local map (orbx_search_local_map,
orbx_search_local_map_batch).

CPU: the oracle's isInFrustum and local-map SearchByProjection against
independent numpy float32/float64 restatements of the same OpenCV 2.4 Mat
semantics.  GPU: the device path
against the oracle, bit-exact on every per-point output (in view, projection,
predicted level, viewing cosine) and on the match vector and counts.
"""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
from local_map_data import make_case, outputs
from oracle_lib import RefExtractor, load
from orb_slam_amd import synth

W, H = 640, 480
f32 = np.float32


@pytest.fixture(scope="module")
def feats():
    frames = synth.sequence(W, H, 2, seed=91)
    ex = RefExtractor(1000)
    return [ex(f) for f in frames]


def ref_lib():
    L = load()
    L.orbx_ref_search_local_map.argtypes = [ctypes.c_void_p]
    L.orbx_ref_search_local_map.restype = ctypes.c_int
    return L


def same(r, g):
    """Bitwise equality of arrays (float outputs compared by bit pattern) or
    equality of scalar counts."""
    r, g = np.asarray(r), np.asarray(g)
    if r.ndim == 0:
        return r == g
    return r.shape == g.shape and np.array_equal(np.ascontiguousarray(r).view(np.uint8),
                                                 np.ascontiguousarray(g).view(np.uint8))


def numpy_in_frustum(a, nlevels=8, scale=1.2):
    """isInFrustum per point, every float32 operation rounded on its own:
    Pc = ((R0 P0 + R1 P1) + R2 P2) + t (OpenCV's small-matrix gemm), invz =
    1.0/PcZ in double, u = fx*PcX*invz + cx, cv::norm / Mat::dot in double."""
    R, t, Ow, cam = a["Rcw"].reshape(3, 3), a["tcw"], a["Ow"], a["cam"]
    sf = [f32(1.0)]
    for _ in range(1, nlevels):
        sf.append(f32(sf[-1] * f32(scale)))
    out = []
    for m in range(len(a["pos"])):
        if a["skip"][m]:
            out.append(None)
            continue
        P = a["pos"][m]
        Pc = [f32(f32(f32(f32(R[r, 0] * P[0]) + f32(R[r, 1] * P[1])) + f32(R[r, 2] * P[2])) + t[r]) for r in range(3)]
        if Pc[2] < 0:
            out.append(None)
            continue
        invz = f32(1.0 / np.float64(Pc[2]))
        u = f32(f32(f32(cam[0] * Pc[0]) * invz) + cam[2])
        v = f32(f32(f32(cam[1] * Pc[1]) * invz) + cam[3])
        if u < 0 or u > W or v < 0 or v > H:
            out.append(None)
            continue
        PO = [f32(P[i] - Ow[i]) for i in range(3)]
        s = 0.0
        for i in range(3):
            s = s + np.float64(PO[i]) * np.float64(PO[i])
        dist = f32(np.sqrt(s))
        dmin, dmax = a["dist"][m]
        if dist < dmin or dist > dmax:
            out.append(None)
            continue
        d = 0.0
        for i in range(3):
            d = d + np.float64(PO[i]) * np.float64(a["normal"][m][i])
        vc = f32(d / np.float64(dist))
        if vc < f32(0.5):
            out.append(None)
            continue
        ratio = f32(dist / dmin)
        lvl = int(np.searchsorted(np.array(sf, np.float32), ratio, side="left"))
        out.append((u, v, min(lvl, nlevels - 1), vc))
    return out


def numpy_search_local(a, want, th, nnratio=0.8):
    """ORBmatcher::SearchByProjection(Frame&, vpMapPoints, th) (src/
    ORBmatcher.cc:49-125) over the points in view: radius RadiusByViewingCos
    (2.5 above a 0.998 cosine, else 4.0; times th unless th == 1) times the
    predicted level's scale; candidates at octaves pred - 1 .. pred without a
    map point (assigned, or matched earlier in this call); best / second with
    their octaves; kept at best <= TH_HIGH unless best and second share an
    octave and best > nnratio * second (float)."""
    from test_match_numpy import Grid, hamming
    from test_proj_numpy import area_levels, scale_factors
    g = Grid(a["kf"], W, H)
    sf = scale_factors()
    taken = a["assigned"].astype(bool).copy()
    out = np.full(len(a["kf"]), -1, np.int64)
    n = 0
    for m, w in enumerate(want):
        if w is None:
            continue
        u, v, lvl, vc = w
        r = f32(2.5) if float(vc) > 0.998 else f32(4.0)
        if th != 1.0:
            r = f32(r * f32(th))
        cand = [c for c in area_levels(g, u, v, f32(r * sf[lvl]), lvl - 1, lvl) if not taken[c]]
        if not cand:
            continue
        dist = hamming(a["desc"][m], a["df"][np.array(cand)])
        best = best2 = 2147483647
        bl = bl2 = -1
        bi = -1
        for c, d in zip(cand, dist):
            d = int(d)
            if d < best:
                best2, best, bl2, bl, bi = best, d, bl, int(a["kf"]["octave"][c]), c
            elif d < best2:
                bl2, best2 = int(a["kf"]["octave"][c]), d
        if best <= 100:
            if bl == bl2 and f32(best) > f32(f32(nnratio) * f32(best2)):
                continue
            taken[bi] = True
            out[bi] = m
            n += 1
    return out, n


@pytest.mark.parametrize("seed,th", [(1, 1.0), (2, 1.0), (3, 5.0)])
def test_oracle_search_local_matches_numpy(feats, seed, th):
    (km, dm), (kf, df) = feats
    a, q = make_case(km, dm, kf, df, W, H, seed, th=th)
    assert ref_lib().orbx_ref_search_local_map(ctypes.byref(q)) == 0
    got, n = numpy_search_local(a, numpy_in_frustum(a), th)
    assert n == q.n_matches > 50
    assert np.array_equal(got, a["matches"].astype(np.int64))


@pytest.mark.parametrize("seed", [1, 2])
def test_oracle_in_frustum_matches_numpy(feats, seed):
    (km, dm), (kf, df) = feats
    a, q = make_case(km, dm, kf, df, W, H, seed)
    assert ref_lib().orbx_ref_search_local_map(ctypes.byref(q)) == 0
    want = numpy_in_frustum(a)
    n_in = 0
    for m, w in enumerate(want):
        assert bool(a["in_view"][m]) == (w is not None), m
        if w is not None:
            n_in += 1
            assert a["proj"][m][0] == w[0] and a["proj"][m][1] == w[1] and a["pred"][m] == w[2] and a["cos"][m] == w[3]
    assert q.n_in_view == n_in > 100
    # every rejection branch is exercised by the generator
    assert n_in < len(want) - int(a["skip"].sum()) - 50
    assert q.n_matches > 50


@pytest.mark.gpu
@pytest.mark.parametrize("seed,th", [(1, 1.0), (2, 5.0), (3, 1.0)])
def test_search_local_map_matches_oracle(feats, seed, th):
    (km, dm), (kf, df) = feats
    ra, rq = make_case(km, dm, kf, df, W, H, seed, th=th)
    ga, gq = make_case(km, dm, kf, df, W, H, seed, th=th)
    assert ref_lib().orbx_ref_search_local_map(ctypes.byref(rq)) == 0
    ctx = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
    assert ox.lib().orbx_search_local_map(ctx.handle, ctypes.byref(gq)) == 0
    ref, got = outputs(ra, rq), outputs(ga, gq)
    for r, g in zip(ref, got):
        assert same(r, g)
    assert gq.n_matches > 0
    ctx.close()


@pytest.mark.gpu
def test_search_local_map_batch_matches_oracle(feats):
    """A batch of frames with different local maps, one with an empty map
    and one with every point skipped (nothing in view: no search), against
    the oracle one query at a time."""
    (km, dm), (kf, df) = feats
    seeds = list(range(10, 16))
    refs = [make_case(km, dm, kf, df, W, H, s, th=5.0 if s % 3 == 0 else 1.0) for s in seeds]
    gots = [make_case(km, dm, kf, df, W, H, s, th=5.0 if s % 3 == 0 else 1.0) for s in seeds]
    for arrs_q in (refs, gots):
        arrs_q[1][1].n_mp = 0                       # empty local map
        arrs_q[2][0]["skip"][:] = 1                 # all skipped
    L = ref_lib()
    for a, q in refs:
        assert L.orbx_ref_search_local_map(ctypes.byref(q)) == 0
    from local_map_data import LocalMapQuery
    arr = (LocalMapQuery * len(gots))(*[q for _, q in gots])
    ctx = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
    assert ox.lib().orbx_search_local_map_batch(ctx.handle, len(gots), arr) == 0
    for b, ((ra, rq), (ga, _)) in enumerate(zip(refs, gots)):
        gq = arr[b]
        ref, got = outputs(ra, rq), outputs(ga, gq)
        for r, g in zip(ref, got):
            assert same(r, g), b
    assert arr[2].n_in_view == 0 and arr[2].n_matches == 0 and arr[1].n_in_view == 0
    ctx.close()
