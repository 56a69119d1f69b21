"""One local-BA problem over several workgroups (k_lba_split, the latency form
of orbx_lba_solve for LocalMapping's single call, src/LocalMapping.cc:83):
bit-identical to the single-workgroup kernel for every workgroup count --
poses, points, outlier decisions, bad points and every LM statistic -- and
at the oracle's bar (tests/test_lba_gpu.py's compare).

The split kernel keeps k_lba_iteration's reductions in their order (the
chi2 / computeScale sums per point, then k_lba_iteration's thread order and
block sum; the reduced system as fixed-point limbs summed exactly over the
workgroups' slabs), so any workgroup count must give the same bits.
"""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
from orb_slam_amd import synth_ba as sb
from test_lba_gpu import compare, run_ref

pytestmark = pytest.mark.gpu


def solve(ctx, prob, wg, abort=None):
    assert ox.lib().orbx_lba_set_workgroups(ctx.handle, wg) == 0
    p, arrs = sb.to_ctypes(prob)
    es = np.zeros(p.n_edges, np.uint8)
    pb = np.zeros(p.n_points, np.uint8)
    st = sb.BAStats()
    ab = None if abort is None else ctypes.byref(ctypes.c_uint8(abort))
    r = ox.lib().orbx_lba_solve(ctx.handle, ctypes.byref(p), 5, 10, ab, es.ctypes.data, pb.ctypes.data,
                                ctypes.byref(st))
    assert r == 0, r
    return arrs, es, pb, st


def same_bits(a, b):
    (aa, ae, ap, ast), (ba, be, bp, bst) = a, b
    for key in ("pose_q", "pose_t", "points"):
        assert np.array_equal(aa[key], ba[key]), key
    assert np.array_equal(ae, be) and np.array_equal(ap, bp)
    for f in ("iterations", "levenberg_trials", "chi2_initial", "chi2_final", "n_outliers"):
        assert list(getattr(ast, f)) == list(getattr(bst, f)), f
    assert ast.not_posdef == bst.not_posdef


@pytest.fixture(scope="module")
def ctx():
    c = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
    yield c
    ox.lib().orbx_lba_set_workgroups(c.handle, 0)
    c.close()


@pytest.mark.parametrize("kw", [dict(n_kf=20, n_points=2000, seed=0), dict(n_kf=20, n_points=2000, seed=77,
                                                                           outlier_frac=0.02),
                                dict(n_kf=10, n_points=600, seed=3, outlier_frac=0.05),
                                dict(n_kf=8, n_points=400, seed=3, normalized=True),
                                dict(n_kf=8, n_points=400, seed=3, info_scale=1e8),
                                dict(n_kf=8, n_points=400, seed=3, near_points=40),
                                dict(n_kf=8, n_points=400, n_fixed_extra=0, seed=7)],
                         ids=["c5", "c5-outliers", "outliers", "normalized", "info-1e8", "near-points", "no-extra-fixed"])
def test_split_equals_one_workgroup(ctx, kw):
    prob = sb.make_problem(**kw)
    one = solve(ctx, prob, 1)
    for wg in (0, 2, 7, 64):
        same_bits(solve(ctx, prob, wg), one)
    compare(run_ref(prob), one)


def test_split_polled_abort_flag(ctx):
    """With an abort flag each iteration is its own launch (the host polls
    between them): the LM state crosses launches through the problem record,
    bit-identical to the unpolled run; a raised flag stops the solve."""
    prob = sb.make_problem(n_kf=12, n_points=900, seed=41)
    base = solve(ctx, prob, 1)
    same_bits(solve(ctx, prob, 0, abort=0), base)
    arrs, es, pb, st = solve(ctx, prob, 0, abort=1)
    assert list(st.iterations) == [0, 0]
    assert np.array_equal(arrs["pose_q"], prob["pose_q"])


def test_split_repeated_calls_reproducible(ctx):
    prob = sb.make_problem(n_kf=20, n_points=2000, seed=5)
    runs = [solve(ctx, prob, 0) for _ in range(3)]
    for r in runs[1:]:
        same_bits(r, runs[0])


def test_workgroup_setting_validates():
    """The setter refuses a null context and counts outside 0..256."""
    assert ox.lib().orbx_lba_set_workgroups(None, 4) == -1
    c = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
    assert ox.lib().orbx_lba_set_workgroups(c.handle, -1) == -1
    assert ox.lib().orbx_lba_set_workgroups(c.handle, 300) == -1
    assert ox.lib().orbx_lba_set_workgroups(c.handle, 16) == 0
    assert ox.lib().orbx_lba_get_workgroups(c.handle) == 16
    c.close()


def _hooks(ctx, fail=0, fallback=1, cap=0, coop=-2):   # coop -2: unchanged
    assert ox.lib().orbx_debug_lba_split(ctx.handle, fail, fallback, cap, coop) == 0


def test_split_capped_at_device_capacity(ctx):
    """The grid barrier needs every workgroup resident: the count is capped
    at the kernel's capacity (occupancy x CUs, here capped by the test hook
    as on a partitioned device), with the same bits."""
    prob = sb.make_problem(n_kf=12, n_points=900, seed=43)
    one = solve(ctx, prob, 1)
    assert ox.lib().orbx_lba_last_workgroups(ctx.handle) == 1
    try:
        _hooks(ctx, cap=5)
        same_bits(solve(ctx, prob, 64), one)
        assert ox.lib().orbx_lba_last_workgroups(ctx.handle) == 5
        _hooks(ctx, cap=1)   # nothing co-resident beyond one: the one-workgroup kernel
        same_bits(solve(ctx, prob, 64), one)
        assert ox.lib().orbx_lba_last_workgroups(ctx.handle) == 1
        _hooks(ctx, cap=0)   # the device's own capacity: the largest setting fits or is capped
        same_bits(solve(ctx, prob, 256), one)
        g = ox.lib().orbx_lba_last_workgroups(ctx.handle)
        assert 2 <= g <= 256
    finally:
        _hooks(ctx, cap=0)


@pytest.mark.parametrize("coop", [0, 1])
def test_split_plain_and_cooperative_launch(ctx, coop):
    prob = sb.make_problem(n_kf=10, n_points=600, seed=44, outlier_frac=0.03)
    one = solve(ctx, prob, 1)
    try:
        _hooks(ctx, coop=coop)
        same_bits(solve(ctx, prob, 0), one)
        assert ox.lib().orbx_lba_last_workgroups(ctx.handle) > 1
    finally:
        _hooks(ctx, coop=0)


def test_split_barrier_timeout_falls_back_to_one_workgroup(ctx):
    """A barrier that times out (workgroups not all resident) makes the call
    run the same solve again on one workgroup: the result equals the
    one-workgroup solve bit for bit."""
    prob = sb.make_problem(n_kf=12, n_points=900, seed=45)
    one = solve(ctx, prob, 1)
    try:
        _hooks(ctx, fail=1)
        same_bits(solve(ctx, prob, 0), one)
        assert ox.lib().orbx_lba_last_workgroups(ctx.handle) == 1
        # the hook is spent: the next solve splits again
        same_bits(solve(ctx, prob, 0), one)
        assert ox.lib().orbx_lba_last_workgroups(ctx.handle) > 1
    finally:
        _hooks(ctx, fail=0)


def test_split_barrier_timeout_without_fallback_leaves_problem_untouched(ctx):
    """With the re-run off the timed-out call returns ORBX_ERR_HIP and
    writes nothing back: poses, points and the output flags keep their
    input values."""
    prob = sb.make_problem(n_kf=12, n_points=900, seed=46)
    assert ox.lib().orbx_lba_set_workgroups(ctx.handle, 0) == 0
    p, arrs = sb.to_ctypes(prob)
    es = np.full(p.n_edges, 7, np.uint8)
    pb = np.full(p.n_points, 7, np.uint8)
    st = sb.BAStats()
    try:
        _hooks(ctx, fail=1, fallback=0)
        r = ox.lib().orbx_lba_solve(ctx.handle, ctypes.byref(p), 5, 10, None, es.ctypes.data, pb.ctypes.data,
                                    ctypes.byref(st))
        assert r == -2
    finally:
        _hooks(ctx, fail=0, fallback=1)
    for key in ("pose_q", "pose_t", "points"):
        assert np.array_equal(arrs[key], np.asarray(prob[key])), key
    assert (es == 7).all() and (pb == 7).all()
    # the context is usable afterwards
    same_bits(solve(ctx, prob, 0), solve(ctx, prob, 1))


def test_split_resident_timeout_falls_back(ctx):
    """orbx_lba_stage / _run / _fetch of one problem (the split kernel) with
    a timed-out barrier: the fetch re-runs the staged problem on one
    workgroup."""
    prob = sb.make_problem(n_kf=12, n_points=900, seed=47)
    one = solve(ctx, prob, 1)
    L = ox.lib()
    assert L.orbx_lba_set_workgroups(ctx.handle, 0) == 0
    p, arrs = sb.to_ctypes(prob)
    arr = (sb.BAProblem * 1)(p)
    es = np.zeros(p.n_edges, np.uint8)
    pb = np.zeros(p.n_points, np.uint8)
    esp = (ctypes.c_void_p * 1)(es.ctypes.data)
    pbp = (ctypes.c_void_p * 1)(pb.ctypes.data)
    st = (sb.BAStats * 1)()
    try:
        _hooks(ctx, fail=1)
        assert L.orbx_lba_stage(ctx.handle, 1, arr) == 0
        assert L.orbx_lba_run(ctx.handle, 5, 10, None) == 0
        assert L.orbx_lba_fetch(ctx.handle, arr, esp, pbp, st) == 0
    finally:
        _hooks(ctx, fail=0)
    same_bits((arrs, es, pb, st[0]), one)


def test_debug_split_hook_validates():
    assert ox.lib().orbx_debug_lba_split(None, 1, 0, 0, -1) == -1
    assert ox.lib().orbx_lba_last_workgroups(None) == -1
