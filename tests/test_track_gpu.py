"""Device-resident Tracking frame (orbx_track_frame: TrackWithMotionModel +
TrackLocalMap, src/Tracking.cc:572-627, 701-752) against the same chain
restated over the oracle's matchers and PoseOptimization
(tests/track_data.py: ref_chain).

The GPU extraction's keypoints are the chain's input on both sides (the
extraction's own parity is tests/test_extract_gpu.py).  In the default
PoseOptimization mode (sums in g2o's order) the whole chain -- matches,
statuses, counts, outlier flags and the final pose -- must equal the
restatement bit for bit.  With the opt-in fast sums
(orbx_pose_set_exact(ctx, 0)) the pose must agree to 1e-5 (north_star's
tolerance for the pose) and everything else exactly.
"""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
import track_data as td

pytestmark = pytest.mark.gpu

W, H = 640, 480
POSE_TOL = 1e-5


@pytest.fixture(scope="module")
def ctx():
    c = ox.Context(nfeatures=1000, max_w=W, max_h=H, slots=4)
    yield c
    c.close()


def features(ctx, img, slot):
    ctx.upload(img, slot)
    ctx.extract(slot, 1)
    ctx.sync()
    return ctx.features(slot)


def px_to_x(px):
    return px * td.DEPTH / float(td.CAM[0])


def setup(ctx, seed, shift, pred_err, **scene_kw):
    last, cur = td.images(W, H, shift, seed)
    kl, dl = features(ctx, last, 0)
    kc, dc = features(ctx, cur, 1)
    scene = td.make_scene(kl, dl, seed, **scene_kw)
    Tpred = td.pose_x(px_to_x(shift + pred_err))
    return last, cur, kl, dl, kc, dc, scene, Tpred


def run(ctx, scene, Tpred, **kw):
    q, keep = td.query(scene, Tpred, **kw)
    rc = ox.lib().orbx_track_frame(ctx.handle, ctypes.byref(q))
    assert rc == 0, ox.ERRORS.get(rc, rc)
    return td.result(q, keep)


def compare(got, exp, exact):
    for k in ("status", "n_cur", "n_motion", "n_pair", "n_after_pose", "n_in_view", "n_local", "n_inliers"):
        assert got[k] == exp[k], (k, got[k], exp[k])
    assert np.array_equal(got["cur_mp"], exp["cur_mp"]), np.count_nonzero(got["cur_mp"] != exp["cur_mp"])
    assert np.array_equal(got["cur_outlier"], exp["cur_outlier"])
    d = np.abs(got["Tcw"] - exp["Tcw"]).max()
    if exact:
        assert np.array_equal(got["Tcw"], exp["Tcw"]), d
    else:
        assert d <= POSE_TOL, d


@pytest.fixture
def pose_mode(ctx):
    yield lambda exact: ox.lib().orbx_pose_set_exact(ctx.handle, int(exact))
    ox.lib().orbx_pose_set_exact(ctx.handle, 1)


@pytest.mark.parametrize("exact", [1, 0])
@pytest.mark.parametrize("seed,shift,pred_err", [(1, 6, 1.5), (2, 10, -2.0), (3, 3, 0.5), (4, 14, 3.0)])
def test_track_frame_matches_oracle_chain(ctx, ref, pose_mode, seed, shift, pred_err, exact):
    pose_mode(exact)
    _, _, kl, dl, kc, dc, scene, Tpred = setup(ctx, seed, shift, pred_err)
    got = run(ctx, scene, Tpred, slot=1, last_view=ox.frame_view(kl, dl, W, H))
    exp = td.ref_chain(ref, kl, dl, kc, dc, scene, Tpred)
    assert exp["status"] == 0 and exp["n_local"] > 0, exp["status"]
    compare(got, exp, exact)


def test_track_frame_motion_failure(ctx, ref, pose_mode):
    """The last frame observes ~15 map points: < 20 motion matches, status
    1, the prediction returned, no PoseOptimization."""
    pose_mode(1)
    _, _, kl, dl, kc, dc, scene, Tpred = setup(ctx, 5, 6, 1.0, observed=0.015)
    got = run(ctx, scene, Tpred, slot=1, last_view=ox.frame_view(kl, dl, W, H))
    exp = td.ref_chain(ref, kl, dl, kc, dc, scene, Tpred)
    assert exp["status"] == 1
    compare(got, exp, True)


@pytest.mark.parametrize("exact", [1, 0])
def test_track_frame_pose_failure(ctx, ref, pose_mode, exact):
    """A prediction 60 px off: the motion search still finds >= 20
    (repetitive texture), PoseOptimization keeps < 10: status 2."""
    pose_mode(exact)
    _, _, kl, dl, kc, dc, scene, Tpred = setup(ctx, 5, 6, 60.0)
    got = run(ctx, scene, Tpred, slot=1, last_view=ox.frame_view(kl, dl, W, H))
    exp = td.ref_chain(ref, kl, dl, kc, dc, scene, Tpred)
    assert exp["status"] == 2 and exp["n_motion"] >= 20
    compare(got, exp, exact)


def test_track_frame_image_and_slot_inputs(ctx, ref, pose_mode):
    """The image path (upload + extraction inside the call) and the last
    frame given as a slot give the results of the slot / view path."""
    pose_mode(1)
    last, cur, kl, dl, kc, dc, scene, Tpred = setup(ctx, 7, 8, 1.0)
    base = run(ctx, scene, Tpred, slot=1, last_view=ox.frame_view(kl, dl, W, H))
    via_image = run(ctx, scene, Tpred, slot=2, image=cur, last_view=ox.frame_view(kl, dl, W, H))
    assert np.array_equal(ctx.features(2)[0], kc)
    via_slot = run(ctx, scene, Tpred, slot=1, last_slot=0)
    exp = td.ref_chain(ref, kl, dl, kc, dc, scene, Tpred)
    for got in (base, via_image, via_slot):
        compare(got, exp, True)


def test_track_sequence_chains_slots(ctx, ref, pose_mode):
    """Three frames: each call tracks the next image against the previous
    call's slot and outputs (cur_mp / cur_outlier become last_mp /
    last_outlier) -- one upload and one read-back per frame."""
    pose_mode(1)
    seed, step = 8, 5
    tex = td.texture(W + 64, H, seed)
    imgs = [np.ascontiguousarray(tex[:, 16 + k * step:16 + k * step + W]) for k in range(3)]
    kl, dl = features(ctx, imgs[0], 0)
    scene = td.make_scene(kl, dl, seed)
    T_last = td.pose_x(0.0)
    slot_last = 0
    for k in (1, 2):
        Tpred = td.pose_x(px_to_x(k * step + 0.7))
        slot = 1 + (k % 2)
        got = run(ctx, scene, Tpred, slot=slot, image=imgs[k], last_slot=slot_last)
        kc, dc = ctx.features(slot)
        exp = td.ref_chain(ref, kl, dl, kc, dc, scene, Tpred)
        compare(got, exp, True)
        assert got["status"] == 0
        # the next frame: this one's map points (outliers dropped, as
        # Tracking::Run does after a good frame, src/Tracking.cc:262-268)
        mp = np.where(got["cur_outlier"] != 0, -1, got["cur_mp"]).astype(np.int32)
        scene = dict(scene, last_mp=mp, last_outlier=np.zeros(len(mp), np.uint8))
        kl, dl, slot_last, T_last = kc, dc, slot, got["Tcw"]


def test_track_frame_last_frame_points_outside_local_map(ctx, ref, pose_mode):
    """n_local_mp: only the first points are the local map searched in the
    frustum step; the last frame's other points still feed the motion
    search."""
    pose_mode(1)
    _, _, kl, dl, kc, dc, scene, Tpred = setup(ctx, 10, 7, 1.0)
    scene["n_local"] = len(kl) // 2
    got = run(ctx, scene, Tpred, slot=1, last_view=ox.frame_view(kl, dl, W, H))
    exp = td.ref_chain(ref, kl, dl, kc, dc, scene, Tpred)
    assert exp["status"] == 0
    compare(got, exp, True)
    assert (got["cur_mp"] >= len(kl) // 2).any()   # motion-only points were matched


@pytest.mark.parametrize("seed,shift,min_octave,observed", [(1, 6, 0, 0.8), (2, 10, 4, 0.8), (3, 3, 0, 0.02),
                                                            (5, 40, 0, 0.8), (6, 6, 0, 0.05)])
def test_track_previous_frame_matches_oracle_chain(ctx, ref, pose_mode, seed, shift, min_octave, observed):
    """mode 1 (TrackPreviousFrame then TrackLocalMap): the window searches,
    the pose from mLastFrame.mTcw, the pair search at 15 (or 50 with too few
    window matches), the pose, the local map -- bit for bit."""
    pose_mode(1)
    last, cur = td.images(W, H, shift, seed)
    kl, dl = features(ctx, last, 0)
    kc, dc = features(ctx, cur, 1)
    scene = td.make_scene(kl, dl, seed, observed=observed)
    Tl = td.pose_x(0.0)
    got = run(ctx, scene, Tl, slot=1, last_view=ox.frame_view(kl, dl, W, H), mode=1, min_octave=min_octave)
    exp = td.ref_chain_prev(ref, kl, dl, kc, dc, scene, Tl, min_octave=min_octave)
    assert exp["status"] == 0
    compare(got, exp, True)
    assert got["n_pair"] == exp["n_pair"]


def test_track_previous_frame_failure(ctx, ref, pose_mode):
    """Almost no map points in the last frame: < 10 window matches, the
    pair search at 50 from mLastFrame.mTcw finds too few: status 3."""
    pose_mode(1)
    last, cur = td.images(W, H, 6, 11)
    kl, dl = features(ctx, last, 0)
    kc, dc = features(ctx, cur, 1)
    scene = td.make_scene(kl, dl, 11, observed=0.004)
    Tl = td.pose_x(0.0)
    got = run(ctx, scene, Tl, slot=1, last_slot=0, mode=1)
    exp = td.ref_chain_prev(ref, kl, dl, kc, dc, scene, Tl)
    assert exp["status"] == 3
    compare(got, exp, True)


def test_track_frame_rejects_bad_queries(ctx):
    _, _, kl, dl, kc, dc, scene, Tpred = setup(ctx, 9, 6, 1.0)
    L = ox.lib()
    for bad in (dict(slot=7), dict(slot=1, last_slot=1), dict(slot=1, last_slot=0, cap=-1),
                dict(slot=1, last_slot=0, nlevels=7), dict(slot=1, last_slot=0, mode=2),
                dict(slot=1, last_slot=0, min_octave=-1)):
        kw = dict(last_view=None if "last_slot" in bad else ox.frame_view(kl, dl, W, H))
        kw.update({k: v for k, v in bad.items() if k in ("slot", "last_slot")})
        q, keep = td.query(scene, Tpred, **kw)
        for k in ("cap", "nlevels", "mode", "min_octave"):
            if k in bad:
                setattr(q, k, bad[k])
        assert L.orbx_track_frame(ctx.handle, ctypes.byref(q)) == -1, bad
    sc = dict(scene, last_mp=np.full(len(kl), len(scene["pos"]), np.int32))   # map index out of range
    q, keep = td.query(sc, Tpred, slot=1, last_view=ox.frame_view(kl, dl, W, H))
    assert L.orbx_track_frame(ctx.handle, ctypes.byref(q)) == -1
