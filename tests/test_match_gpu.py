"""GPU parity of ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:
598-713) on consecutive frames of a synthetic sequence.  The oracle runs on
the GPU-extracted features (themselves checked bit-exact in
test_extract_gpu.py), so this isolates the greedy matcher replay."""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
from orb_slam_amd import synth
from oracle_lib import load, ptr

pytestmark = pytest.mark.gpu


def ref_search_init(L, k1, d1, k2, d2, w, h, window=100, nnratio=0.9, check_ori=True):
    F1 = ox.frame_view(k1, d1, w, h)
    F2 = ox.frame_view(k2, d2, w, h)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32).copy()
    m12 = np.zeros(len(k1), np.int32)
    nm = ctypes.c_int()
    assert L.orbx_ref_search_for_initialization(ctypes.byref(F1), ctypes.byref(F2), ptr(prev), ptr(m12),
                                                window, nnratio, int(check_ori), ctypes.byref(nm)) == 0
    return m12, nm.value


@pytest.mark.parametrize("n,seq_len", [(1000, 8), (2000, 5)])
def test_match_prev_matches_oracle(n, seq_len):
    w, h = 640, 480
    frames = synth.sequence(w, h, seq_len, seed=21 + n)
    ctx = ox.Context(nfeatures=n, max_w=w, max_h=h, slots=seq_len)
    ctx.upload(frames)
    ctx.extract(0, seq_len)
    ctx.match_prev(0, seq_len, seq_len, window=100, nnratio=0.9, check_ori=True)
    ctx.sync()
    L = load()
    feats = [ctx.features(s) for s in range(seq_len)]
    total = 0
    for s in range(seq_len):
        p = s - 1 if s % seq_len else s + seq_len - 1
        k1, d1 = feats[p]
        k2, d2 = feats[s]
        rm, rn = ref_search_init(L, k1, d1, k2, d2, w, h)
        gm, gn = ctx.matches(s)
        assert gn == rn, (s, gn, rn)
        assert np.array_equal(gm[:len(k1)], rm), (s, np.count_nonzero(gm[:len(k1)] != rm))
        total += gn
    assert total > 0
    ctx.close()


@pytest.mark.parametrize("window,nnratio,check_ori", [(50, 0.6, True), (150, 0.75, False), (20, 0.9, False)])
def test_match_prev_parameters(window, nnratio, check_ori):
    """The batched device path with ORBmatcher(nnratio, checkOri) and window
    sizes other than Tracking's (src/Tracking.cc:361: 0.9, true, 100)."""
    w, h, n, seq_len = 640, 480, 1000, 6
    frames = synth.sequence(w, h, seq_len, seed=40 + window)
    ctx = ox.Context(nfeatures=n, max_w=w, max_h=h, slots=seq_len)
    ctx.upload(frames)
    ctx.extract(0, seq_len)
    ctx.match_prev(0, seq_len, seq_len, window=window, nnratio=nnratio, check_ori=check_ori)
    ctx.sync()
    L = load()
    feats = [ctx.features(s) for s in range(seq_len)]
    for s in range(seq_len):
        p = s - 1 if s % seq_len else s + seq_len - 1
        k1, d1 = feats[p]
        k2, d2 = feats[s]
        rm, rn = ref_search_init(L, k1, d1, k2, d2, w, h, window, nnratio, check_ori)
        gm, gn = ctx.matches(s)
        assert gn == rn, (s, gn, rn)
        assert np.array_equal(gm[:len(k1)], rm), (s, np.count_nonzero(gm[:len(k1)] != rm))
    ctx.close()


@pytest.mark.parametrize("th_low,nnratio", [(40, 0.8), (80, 0.95)])
def test_match_bf_prev_parameters(th_low, nnratio):
    w, h, n, seq_len = 640, 480, 1000, 3
    frames = synth.sequence(w, h, seq_len, seed=th_low)
    ctx = ox.Context(nfeatures=n, max_w=w, max_h=h, slots=seq_len)
    ctx.upload(frames)
    ctx.extract(0, seq_len)
    ctx.match_bf_prev(0, seq_len, seq_len, th_low=th_low, nnratio=nnratio)
    ctx.sync()
    L = load()
    feats = [ctx.features(s) for s in range(seq_len)]
    for s in range(seq_len):
        p = s - 1 if s % seq_len else s + seq_len - 1
        dA, dB = feats[p][1], feats[s][1]
        bi, b1, b2 = (np.zeros(len(dA), np.int32) for _ in range(3))
        L.orbx_ref_hamming_bf(ptr(dA), len(dA), ptr(dB), len(dB), ptr(bi), ptr(b1), ptr(b2))
        want = np.where((b1 <= th_low) & (b1.astype(np.float32) < b2.astype(np.float32) * np.float32(nnratio)), bi, -1)
        gm, gn = ctx.matches(s)
        assert np.array_equal(gm[:len(dA)], want)
    ctx.close()


@pytest.mark.parametrize("n", [150, 300, 1000])
def test_match_bf_prev_ragged_counts(n):
    """k_match_bf_prev_mfma at keypoint counts off its 32-wide tiles and
    128-candidate chunks, and with an empty frame (flat: no FAST corners) on
    either side of a pair."""
    w, h, seq_len = 640, 480, 4
    frames = synth.sequence(w, h, seq_len, seed=11 + n)
    frames[1][:, 200:] = 128   # texture on a third of the frame: a ragged count
    frames[2] = 128
    ctx = ox.Context(nfeatures=n, max_w=w, max_h=h, slots=seq_len)
    ctx.upload(frames)
    ctx.extract(0, seq_len)
    ctx.match_bf_prev(0, seq_len, seq_len, th_low=50, nnratio=0.9)
    ctx.sync()
    L = load()
    feats = [ctx.features(s) for s in range(seq_len)]
    assert len(feats[2][1]) == 0 and 0 < len(feats[1][1]) <= n
    for s in range(seq_len):
        p = s - 1 if s % seq_len else s + seq_len - 1
        dA, dB = feats[p][1], feats[s][1]
        gm, gn = ctx.matches(s)
        if len(dA) == 0 or len(dB) == 0:
            assert gn == 0
            continue
        bi, b1, b2 = (np.zeros(len(dA), np.int32) for _ in range(3))
        L.orbx_ref_hamming_bf(ptr(dA), len(dA), ptr(dB), len(dB), ptr(bi), ptr(b1), ptr(b2))
        want = np.where((b1 <= 50) & (b1.astype(np.float32) < b2.astype(np.float32) * np.float32(0.9)), bi, -1)
        assert np.array_equal(gm[:len(dA)], want)
        assert gn == int((want >= 0).sum())
    ctx.close()


def test_match_bf_prev_matches_oracle():
    """Device-resident brute-force pairs (C3) against the oracle's all-pairs
    best/second + the acceptance rule."""
    w, h, n, seq_len = 640, 480, 1000, 4
    frames = synth.sequence(w, h, seq_len, seed=5)
    ctx = ox.Context(nfeatures=n, max_w=w, max_h=h, slots=seq_len)
    ctx.upload(frames)
    ctx.extract(0, seq_len)
    ctx.match_bf_prev(0, seq_len, seq_len, th_low=50, nnratio=0.9)
    ctx.sync()
    L = load()
    feats = [ctx.features(s) for s in range(seq_len)]
    for s in range(seq_len):
        p = s - 1 if s % seq_len else s + seq_len - 1
        dA, dB = feats[p][1], feats[s][1]
        bi, b1, b2 = (np.zeros(len(dA), np.int32) for _ in range(3))
        L.orbx_ref_hamming_bf(ptr(dA), len(dA), ptr(dB), len(dB), ptr(bi), ptr(b1), ptr(b2))
        want = np.where((b1 <= 50) & (b1.astype(np.float32) < b2.astype(np.float32) * np.float32(0.9)), bi, -1)
        gm, gn = ctx.matches(s)
        assert np.array_equal(gm[:len(dA)], want)
        assert gn == int((want >= 0).sum()) and gn > 0
    ctx.close()


@pytest.mark.parametrize("mode,seq_len", [("init", 64), ("init", 16), ("bf", 64)])
def test_extract_match_pipeline_equals_separate_calls(mode, seq_len):
    """orbx_dev_extract_match (two-stream pipelined, pairs straddling the
    halves matched after the join) gives exactly the separate calls' result."""
    w, h, B = 640, 480, 64
    frames = synth.sequence(w, h, B, seed=13)
    ctx = ox.Context(nfeatures=1000, max_w=w, max_h=h, slots=B)
    ctx.upload(frames)
    ctx.extract_match(0, B, seq_len, mode=mode)
    ctx.sync()
    piped = [ctx.matches(s) for s in range(B)]
    feats = [ctx.features(s) for s in range(B)]
    ctx.set_split(False)
    ctx.extract(0, B)
    if mode == "init":
        ctx.match_prev(0, B, seq_len)
    else:
        ctx.match_bf_prev(0, B, seq_len)
    ctx.sync()
    for s in range(B):
        m, n = ctx.matches(s)
        k, d = ctx.features(s)
        assert np.array_equal(k.view(np.uint8), feats[s][0].view(np.uint8)) and np.array_equal(d, feats[s][1])
        assert n == piped[s][1] and np.array_equal(m[:len(k)], piped[s][0][:len(k)]), s
    ctx.close()


@pytest.mark.parametrize("mode", ["init", "bf"])
def test_async_extract_match_alternating_slots(mode):
    """Asynchronous matching (orbx_dev_set_async_match): batches alternating
    between two slot ranges, each batch's matching overlapping the next
    batch's extraction, give the synchronous calls' results."""
    w, h, B = 640, 480, 32
    frames = synth.sequence(w, h, 2 * B, seed=17)
    ctx = ox.Context(nfeatures=1000, max_w=w, max_h=h, slots=2 * B)
    ctx.upload(frames)
    ctx.set_async_match(True)
    for it in range(3):
        ctx.extract_match((it % 2) * B, B, B, mode=mode)
    ctx.sync()
    got = [ctx.matches(s) for s in range(2 * B)]
    ctx.set_async_match(False)
    for first in (0, B):
        ctx.extract(first, B)
        if mode == "init":
            ctx.match_prev(first, B, B)
        else:
            ctx.match_bf_prev(first, B, B)
    ctx.sync()
    for s in range(2 * B):
        m, n = ctx.matches(s)
        k, _ = ctx.features(s)
        assert n == got[s][1] and np.array_equal(m[:len(k)], got[s][0][:len(k)]), s
    ctx.close()


def test_async_pipeline_reused_slots_odd_batch():
    """The two-stream extract+match pipeline with an odd batch (halves of 18
    and 19 frames), the same slot range extracted again while its previous
    match is pending, and new frames uploaded between pipelined calls: every
    slot's keypoints, descriptors and matches equal the synchronous path's."""
    w, h, B = 320, 240, 37
    seqs = [synth.sequence(w, h, B, seed=s) for s in (41, 42)]
    ctx = ox.Context(nfeatures=500, max_w=w, max_h=h, slots=B)

    def snapshot():
        return [(*ctx.features(s), *ctx.matches(s)) for s in range(B)]

    def reference(frames):
        ctx.set_async_match(False)
        ctx.upload(frames)
        ctx.extract(0, B)
        ctx.match_prev(0, B, B)
        ctx.sync()
        return snapshot()

    want = [reference(f) for f in seqs]
    ctx.set_async_match(True)
    ctx.upload(seqs[0])
    ctx.extract_match(0, B, B)
    ctx.extract_match(0, B, B)      # same slots: waits for the pending match
    ctx.upload(seqs[1])             # new frames while nothing is pending any more
    ctx.extract_match(0, B, B)
    ctx.sync()
    got = snapshot()
    for s in range(B):
        gk, gd, gm, gn = got[s]
        rk, rd, rm, rn = want[1][s]
        assert np.array_equal(gk, rk) and np.array_equal(gd, rd), s
        assert gn == rn and np.array_equal(gm[:len(gk)], rm[:len(rk)]), s
    ctx.close()


@pytest.mark.parametrize("seed", range(8))
def test_match_prev_random_sizes(seed):
    """SearchForInitialization on the device path for random frame sizes and
    feature counts (the frame grid's cell size follows the image bounds)."""
    r = np.random.default_rng(300 + seed)
    w, h = int(r.integers(120, 900)), int(r.integers(100, 700))
    n, seq_len = int(r.integers(100, 2500)), 4
    window = int(r.choice([30, 100, 200]))
    frames = synth.sequence(w, h, seq_len, seed=400 + seed)
    try:
        ctx = ox.Context(nfeatures=n, max_w=w, max_h=h, slots=seq_len)
    except ox.OrbxError as e:
        # a level whose cell grid is empty: the reference divides by zero
        # (src/ORBextractor.cc:533-541); the oracle refuses it as well
        from oracle_lib import RefExtractor
        with pytest.raises(AssertionError):
            RefExtractor(n)(frames[0])
        assert e.code == -4
        return
    ctx.upload(frames)
    ctx.extract(0, seq_len)
    ctx.match_prev(0, seq_len, seq_len, window=window, nnratio=0.9, check_ori=True)
    ctx.sync()
    L = load()
    feats = [ctx.features(s) for s in range(seq_len)]
    for s in range(seq_len):
        p = s - 1 if s % seq_len else s + seq_len - 1
        k1, d1 = feats[p]
        k2, d2 = feats[s]
        rm, rn = ref_search_init(L, k1, d1, k2, d2, w, h, window)
        gm, gn = ctx.matches(s)
        assert gn == rn, (s, gn, rn)
        assert np.array_equal(gm[:len(k1)], rm)
    ctx.close()
