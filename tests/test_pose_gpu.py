"""GPU Optimizer::PoseOptimization (src/Optimizer.cc:154-285) through the C
ABI against the FP64 CPU restatement (oracle/ref_pose.cpp).

Default mode (sums sequentially in g2o's active-edge order, one frame on the
eight-wavefront kernel, batches a wavefront per frame): the whole LM
trajectory must equal the restatement's -- iterations, trials and outliers of
every round, the final chi2 of each round, the inlier count and the pose bit
for bit, for every batch size.

The opt-in fast sums (orbx_pose_set_exact(ctx, 0): lane-strided partials
through a fixed DPP tree) are held to north_star's pose tolerance: mTcw within
1e-5 (absolute, all entries), mvbOutlier and the inlier count identical.
"""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
from orb_slam_amd import synth_pose as sp
from test_pose_oracle import ref_pose

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-5


@pytest.fixture(scope="module")
def ctx():
    c = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
    yield c
    c.close()


def gpu_pose(ctx, frames):
    structs, arrs = zip(*[sp.to_ctypes(fr) for fr in frames])
    structs = list(structs)
    n, st = ctx.pose_optimization(structs)
    return [(sp.pose_of(structs[k]), arrs[k]["outlier"], int(n[k]), st[k]) for k in range(len(frames))]


def compare_exact(ref, gpu):
    rT, rout, rn, rst = ref
    gT, gout, gn, gst = gpu
    assert gst.rounds == rst.rounds
    assert list(gst.iterations) == list(rst.iterations)
    assert list(gst.levenberg_trials) == list(rst.levenberg_trials)
    assert list(gst.n_bad) == list(rst.n_bad)
    assert gst.not_posdef == rst.not_posdef
    assert list(gst.chi2_final) == list(rst.chi2_final)
    assert np.array_equal(gout, rout) and gn == rn
    assert np.array_equal(gT, rT), np.abs(gT - rT).max()


def compare_fast(ref, gpu):
    rT, rout, rn, rst = ref
    gT, gout, gn, gst = gpu
    d = np.abs(gT - rT).max()
    assert d <= POSE_TOL, d
    assert np.array_equal(gout, rout), np.count_nonzero(gout != rout)
    assert gn == rn
    return d


CASES = [dict(n_kp=1000, seed=0), dict(n_kp=1000, seed=1, outlier_frac=0.2), dict(n_kp=200, seed=2, outlier_frac=0.3),
         dict(n_kp=3000, seed=3, mp_frac=0.9), dict(n_kp=64, seed=4), dict(n_kp=12, seed=5, mp_frac=0.6),
         dict(n_kp=1000, seed=6, pix_noise=0.0, outlier_frac=0.0), dict(n_kp=500, seed=7, outlier_frac=0.9)]
EXACT_CASES = CASES + [dict(n_kp=1000, seed=s, outlier_frac=0.1) for s in range(20, 36)]


@pytest.fixture()
def fast_ctx(ctx):
    assert ox.lib().orbx_pose_set_exact(ctx.handle, 0) == 0
    assert ox.lib().orbx_pose_get_exact(ctx.handle) == 0
    yield ctx
    assert ox.lib().orbx_pose_set_exact(ctx.handle, 1) == 0


def test_pose_default_is_exact(ctx):
    assert ox.lib().orbx_pose_get_exact(ctx.handle) == 1


@pytest.mark.parametrize("case", EXACT_CASES, ids=[f"n{c['n_kp']}_s{c['seed']}" for c in EXACT_CASES])
def test_pose_matches_oracle(ctx, case):
    """One call (the eight-wavefront kernel): the LM trajectory of every
    round equals the restatement's -- counts, outliers, per-round chi2 and
    pose; entries without a map point stay untouched."""
    fr = sp.make_frame(**case)
    fr["outlier"][:] = 7
    compare_exact(ref_pose(fr), gpu_pose(ctx, [fr])[0])


@pytest.mark.parametrize("case", CASES, ids=[f"n{c['n_kp']}_s{c['seed']}" for c in CASES])
def test_pose_fast_sums_within_tolerance(fast_ctx, case):
    fr = sp.make_frame(**case)
    fr["outlier"][:] = 7
    compare_fast(ref_pose(fr), gpu_pose(fast_ctx, [fr])[0])


def test_pose_no_map_points_and_empty_frame(ctx):
    a = sp.make_frame(n_kp=40, seed=8)
    a["has_mp"][:] = 0
    a["outlier"][:] = 3
    b = sp.make_frame(n_kp=0, seed=9)
    for ref, gpu in zip([ref_pose(a), ref_pose(b)], gpu_pose(ctx, [a, b])):
        compare_exact(ref, gpu)


def test_pose_batch_mixed_sizes(ctx):
    """A batch (a wavefront per frame): bit for bit the restatement, so the
    same frame gives the same result alone and in a batch."""
    rng = np.random.default_rng(1)
    frames = [sp.make_frame(n_kp=int(rng.integers(5, 1500)), seed=300 + k, outlier_frac=float(rng.uniform(0, 0.3)))
              for k in range(23)]
    batch = gpu_pose(ctx, frames)
    for fr, g in zip(frames, batch):
        compare_exact(ref_pose(fr), g)
    alone = gpu_pose(ctx, frames[:1])[0]
    assert np.array_equal(alone[0], batch[0][0]) and np.array_equal(alone[1], batch[0][1])


def test_pose_batch_active_lists(ctx):
    """The batch kernel walks each later robust round's active edges from a
    list of at most 2048 (kPoseActCap) and every edge above that: frames
    around and over the cap, mostly-outlier and outlier-free frames, bit for
    bit the restatement."""
    cases = [dict(n_kp=3000, seed=400, mp_frac=0.9, outlier_frac=0.2),   # ~2700 edges: no list
             dict(n_kp=2200, seed=401, mp_frac=0.93, outlier_frac=0.1),  # ~2050 edges: at the cap
             dict(n_kp=2000, seed=402, mp_frac=0.9, outlier_frac=0.15),
             dict(n_kp=500, seed=403, outlier_frac=0.9),
             dict(n_kp=700, seed=404, pix_noise=0.0, outlier_frac=0.0),
             dict(n_kp=65, seed=405, outlier_frac=0.5)]
    frames = [sp.make_frame(**c) for c in cases]
    assert any(int(fr["has_mp"].sum()) > 2048 for fr in frames)
    for fr, g in zip(frames, gpu_pose(ctx, frames)):
        compare_exact(ref_pose(fr), g)


def test_pose_degenerate_edge_takes_the_division_path(ctx):
    """The per-edge terms divide through shared reciprocals only where the
    camera-frame point keeps v_div_scale from rescaling (orbx_pose.hip
    div_safe); a point on the camera plane (z = 0) takes the original
    divisions, on one lane of a wave whose other lanes take the fast path.
    Its infinite error makes every chi2 NaN, as in the restatement, so every
    trial is rejected there too: the same counts, outliers and pose (chi2
    compared NaN-aware), alone and in a batch."""
    fr = sp.make_frame(n_kp=300, seed=500)
    fr["Tcw"] = np.eye(4, dtype=np.float32)           # pc = X exactly (identity quaternion, t = 0)
    k = int(np.nonzero(fr["has_mp"])[0][5])
    fr["mp_xyz"][k] = [0.5, -0.25, 0.0]               # z = 0: outside div_safe
    other = sp.make_frame(n_kp=400, seed=501)
    ref = ref_pose(fr)
    for got in (gpu_pose(ctx, [fr])[0], gpu_pose(ctx, [fr, other])[0]):
        rT, rout, rn, rst = ref
        gT, gout, gn, gst = got
        assert gst.rounds == rst.rounds
        assert list(gst.iterations) == list(rst.iterations)
        assert list(gst.levenberg_trials) == list(rst.levenberg_trials)
        assert list(gst.n_bad) == list(rst.n_bad)
        assert np.array_equal(np.array(gst.chi2_final), np.array(rst.chi2_final), equal_nan=True)
        assert np.array_equal(gout, rout) and gn == rn
        assert np.array_equal(gT, rT, equal_nan=True)


def test_pose_fast_sums_batch_mixed_sizes(fast_ctx):
    rng = np.random.default_rng(0)
    frames = [sp.make_frame(n_kp=int(rng.integers(5, 1500)), seed=100 + k, outlier_frac=float(rng.uniform(0, 0.3)))
              for k in range(37)]
    for fr, g in zip(frames, gpu_pose(fast_ctx, frames)):
        compare_fast(ref_pose(fr), g)


def test_pose_staged_rerun_is_idempotent(ctx):
    frames = [sp.make_frame(n_kp=800, seed=200 + k) for k in range(9)]
    keep = [sp.to_ctypes(fr) for fr in frames]           # arrays the structs point into
    structs = [k[0] for k in keep]
    ctx.pose_stage(structs)
    ctx.pose_run()
    arr1, n1, _ = ctx.pose_fetch()
    T1 = [sp.pose_of(arr1[k]) for k in range(len(frames))]
    ctx.pose_run()
    ctx.pose_run()
    arr2, n2, _ = ctx.pose_fetch()
    for k in range(len(frames)):
        assert np.array_equal(T1[k], sp.pose_of(arr2[k]))
    assert np.array_equal(n1, n2)
    for k, fr in enumerate(frames):
        rT, rout, rn, _ = ref_pose(fr)
        assert np.array_equal(T1[k], rT) and n1[k] == rn


def test_pose_rejects_bad_octave(ctx):
    fr = sp.make_frame(n_kp=20, seed=10)
    fr["octave"][fr["has_mp"].astype(bool).nonzero()[0][0]] = 8
    p, arrs = sp.to_ctypes(fr)
    n = ctypes.c_int()
    assert ox.lib().orbx_pose_optimization(ctx.handle, ctypes.byref(p), ctypes.byref(n), None) == -1


def test_pose_exact_setter_validates():
    assert ox.lib().orbx_pose_set_exact(None, 1) == -1
    c = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
    assert ox.lib().orbx_pose_get_exact(c.handle) == 1
    assert ox.lib().orbx_pose_set_exact(c.handle, 2) == -1
    assert ox.lib().orbx_pose_set_exact(c.handle, -1) == -1
    c.close()
