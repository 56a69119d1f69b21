"""Parity at the exact shapes bench.py measures.

The other GPU tests stop at 64-frame batches; the bench runs
* C2: 1024 frames of 640x480 / 1000 kp per step, two slot ranges (2 x 1024
  slots), asynchronous matching (orbx_dev_set_async_match), the default
  three-part extraction pipeline, ranges alternating between steps;
* C3: 1920x1080 / 2000 kp, 128 frames per step, brute-force pairs on the
  device (k_match_bf_prev), same pipeline;
* C5: 256 resident local-BA problems of 20 KF x 2000 MP (orbx_lba_stage /
  run / fetch).
Each test drives that exact call sequence and checks sampled units against
the oracle (ORBextractor::operator() src/ORBextractor.cc:718-779,
SearchForInitialization src/ORBmatcher.cc:598-713, the brute-force rule of
:640-654, LocalBundleAdjustment src/Optimizer.cc:287-536), including the
pipeline's part boundaries, plus every slot against the synchronous device
path (bit-exact).
"""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
from orb_slam_amd import synth, synth_ba as sb
from oracle_lib import RefExtractor, load, ptr

pytestmark = pytest.mark.gpu


def part_bounds(count, ways):
    """First and last slot of each pipeline part (orbx_extract.hip: part i
    covers [count*i/ways, count*(i+1)/ways))."""
    out = []
    for i in range(ways):
        lo, hi = count * i // ways, count * (i + 1) // ways
        out += [lo, hi - 1]
    return out


def ref_init(L, k1, d1, k2, d2, w, h):
    F1, F2 = ox.frame_view(k1, d1, w, h), ox.frame_view(k2, d2, w, h)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32).copy()
    m = np.zeros(len(k1), np.int32)
    nm = ctypes.c_int()
    assert L.orbx_ref_search_for_initialization(ctypes.byref(F1), ctypes.byref(F2), ptr(prev), ptr(m), 100, 0.9, 1,
                                                ctypes.byref(nm)) == 0
    return m, nm.value


def ref_bf(L, dA, dB, th_low=50, nnratio=0.9):
    bi, b1, b2 = (np.zeros(len(dA), np.int32) for _ in range(3))
    L.orbx_ref_hamming_bf(ptr(dA), len(dA), ptr(dB), len(dB), ptr(bi), ptr(b1), ptr(b2))
    want = np.where((b1 <= th_low) & (b1.astype(np.float32) < b2.astype(np.float32) * np.float32(nnratio)), bi, -1)
    return want, int((want >= 0).sum())


def run_bench_pipeline(w, h, nf, B, mode, split_ways=None, steps=3, seed=2000, era=None):
    """bench.py run_frames: slots = 2B, both ranges uploaded with the same
    sequence, async matching, steps alternating the ranges.  era: retainBest's
    libstdc++ era (orbx_set_nth_pivot), None = the library default."""
    frames = synth.sequence(w, h, B, seed=seed)
    ctx = ox.Context(nfeatures=nf, max_w=w, max_h=h, slots=2 * B)
    if era is not None:
        ctx.set_nth_pivot(era)
    ctx.upload(frames, first=0)
    ctx.upload(frames, first=B)
    if split_ways:
        assert ox.lib().orbx_dev_set_split(ctx.handle, split_ways) == 0
    ctx.set_async_match(True)
    for it in range(steps):
        ctx.extract_match((it % 2) * B, B, B, mode=mode, window=100, th_low=50, nnratio=0.9, check_ori=True)
    ctx.sync()
    return frames, ctx


def snapshot(ctx, slots):
    return {s: (*ctx.features(s), *ctx.matches(s)) for s in slots}


def check_against_sync(ctx, B, mode, got):
    """Re-run both ranges through the synchronous, unsplit device path and
    require every slot to be bit-identical to the pipelined result."""
    ctx.set_async_match(False)
    ctx.set_split(False)
    for first in (0, B):
        ctx.extract(first, B)
        if mode == "init":
            ctx.match_prev(first, B, B)
        else:
            ctx.match_bf_prev(first, B, B)
    ctx.sync()
    for s, (gk, gd, gm, gn) in got.items():
        k, d = ctx.features(s)
        m, n = ctx.matches(s)
        assert np.array_equal(k.view(np.uint8), gk.view(np.uint8)) and np.array_equal(d, gd), s
        assert n == gn and np.array_equal(m[:len(k)], gm[:len(gk)]), s


def check_against_oracle(frames, got, B, nf, w, h, mode, sample, era=1):
    ex = RefExtractor(nf, nth_pivot=era)
    L = load()
    ref = {}
    for s in sorted(set(sample) | {(s % B - 1) % B for s in sample}):
        ref[s] = ex(frames[s])
    for s in sample:
        f = s % B
        p = (f - 1) % B
        rk, rd = ref[f]
        for base in (0, B):
            gk, gd, gm, gn = got[base + f]
            assert len(gk) > 0 and np.array_equal(gk, rk) and np.array_equal(gd, rd), ("extract", base + f)
        pk, pd = ref[p]
        if mode == "init":
            rm, rn = ref_init(L, pk, pd, rk, rd, w, h)
        else:
            rm, rn = ref_bf(L, pd, rd)
        for base in (0, B):
            gk, gd, gm, gn = got[base + f]
            assert gn == rn and np.array_equal(gm[:len(pk)], rm), ("match", base + f, gn, rn)
        assert rn > 0


@pytest.mark.parametrize("era", [None, 0], ids=["default-gcc48", "gcc49"])
def test_c2_bench_pipeline_1024_three_parts(era):
    """C2 exactly as benched: 1024-frame steps, three parts, async matching,
    three steps alternating the two slot ranges.  Twelve frames (the part
    boundaries 0/340/341/681/682/1023 and six interior ones) against the
    oracle in both ranges; all 2048 slots against the synchronous path.  In
    both libstdc++ eras of retainBest: the default (GCC 4.6 .. 4.8, the
    bench's) and GCC >= 4.9."""
    w, h, nf, B = 640, 480, 1000, 1024
    frames, ctx = run_bench_pipeline(w, h, nf, B, "init", era=era)
    assert ox.lib().orbx_get_nth_pivot(ctx.handle) == (1 if era is None else era)
    got = snapshot(ctx, range(2 * B))
    sample = sorted(set(part_bounds(B, 3)) | {1, 170, 299, 300, 511, 900})
    check_against_oracle(frames, got, B, nf, w, h, "init", sample, era=1 if era is None else era)
    check_against_sync(ctx, B, "init", got)
    ctx.close()


@pytest.mark.parametrize("B,ways", [(48, 3), (64, 4), (97, 4), (96, 2)])
def test_async_pipeline_parts(B, ways):
    """the 3- and 4-part asynchronous pipelines at small batches
    (parts on xstreams[0]/[1], the ev_part_fast release chain over more than
    two streams, the match stream joining every part), alternating slot
    ranges, plus the same range re-extracted while its match is pending."""
    w, h, nf = 320, 240, 500
    frames, ctx = run_bench_pipeline(w, h, nf, B, "init", split_ways=ways, steps=4)
    # a fifth call on the range whose match may still be pending
    ctx.extract_match(B, B, B, mode="init")
    ctx.sync()
    got = snapshot(ctx, range(2 * B))
    sample = sorted(set(part_bounds(B, ways)))
    check_against_oracle(frames, got, B, nf, w, h, "init", sample)
    check_against_sync(ctx, B, "init", got)
    ctx.close()


@pytest.mark.parametrize("era", [None, 0], ids=["default-gcc48", "gcc49"])
def test_c3_bench_pipeline_1080p_bf(era):
    """C3 exactly as benched: 1920x1080 / 2000 kp, 128-frame steps, three
    parts, async device brute-force pairs (k_match_bf_prev) at full size,
    alternating ranges; part boundaries and frame 0 (matched against the
    cyclic predecessor 127) against the oracle, in both retainBest eras."""
    w, h, nf, B = 1920, 1080, 2000, 128
    frames, ctx = run_bench_pipeline(w, h, nf, B, "bf", era=era)
    got = snapshot(ctx, range(2 * B))
    sample = sorted(set(part_bounds(B, 3)) | {64})
    check_against_oracle(frames, got, B, nf, w, h, "bf", sample, era=1 if era is None else era)
    check_against_sync(ctx, B, "bf", got)
    ctx.close()


def test_c5_resident_batch_256_vs_oracle():
    """C5 exactly as benched: 256 resident problems (20 KF x 2000 MP, the
    bench's distinct problems repeated), staged once, two runs, fetched;
    one copy of every distinct problem against the oracle (poses 1e-5,
    points 1e-4, identical outlier decisions and LM trajectories) and the
    repeated copies identical to each other."""
    from test_lba_gpu import POINT_TOL, POSE_TOL, run_ref
    P, U = 256, 8
    uniq = [sb.make_problem(n_kf=20, n_points=2000, seed=5000 * 1000 + i) for i in range(U)]
    probs = [uniq[i % U] for i in range(P)]
    L = ox.lib()
    ctx = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
    work = [sb.to_ctypes(pr) for pr in probs]
    arr = (sb.BAProblem * P)(*[c[0] for c in work])
    assert L.orbx_lba_stage(ctx.handle, P, arr) == 0
    for _ in range(2):
        assert L.orbx_lba_run(ctx.handle, 5, 10, None) == 0
    es = [np.zeros(c[0].n_edges, np.uint8) for c in work]
    pb = [np.zeros(c[0].n_points, np.uint8) for c in work]
    esp = (ctypes.c_void_p * P)(*[e.ctypes.data for e in es])
    pbp = (ctypes.c_void_p * P)(*[b.ctypes.data for b in pb])
    st = (sb.BAStats * P)()
    assert L.orbx_lba_fetch(ctx.handle, arr, esp, pbp, st) == 0
    for u in range(U):
        ra, res, rpb, rst = run_ref(uniq[u])
        for i in (u, u + U * 17, P - U + u):
            a = work[i][1]
            assert np.abs(a["pose_q"] - ra["pose_q"]).max() <= POSE_TOL, (u, i)
            assert np.abs(a["pose_t"] - ra["pose_t"]).max() <= POSE_TOL, (u, i)
            assert np.abs(a["points"] - ra["points"]).max() <= POINT_TOL, (u, i)
            assert np.array_equal(es[i], res) and np.array_equal(pb[i], rpb), (u, i)
            assert list(st[i].iterations) == list(rst.iterations), (u, i)
            assert list(st[i].levenberg_trials) == list(rst.levenberg_trials), (u, i)
            assert list(st[i].n_outliers) == list(rst.n_outliers), (u, i)
    ctx.close()
