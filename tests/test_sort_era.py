"""retainBest's libstdc++ era ("unpinned semantics": sort era).

KeyPointsFilter::retainBest (src/ORBextractor.cc:683, :699) keeps the first
n entries of std::nth_element's permutation.  libstdc++ changed
__introselect's pivot step in GCC 4.9 (PR libstdc++/58437): the median of
(first + 1, mid, last - 1) swapped into *first, where GCC 4.6 .. 4.8 -- the
compilers of the reference's era -- moved the median of (first, mid,
last - 1) to *first.  With integer FAST scores ties at the retain boundary
are common, so which tied corners survive, and their order, depend on it.

The oracle restates nth_element with either pivot step
(oracle/ref_extract.cpp libstdcxx_nth_element); these tests pin the
restatement against this image's std::nth_element (GCC 11.4, the newer
rule), check both eras produce valid nth_element results, and measure how
often the choice changes a 640x480 extraction.  The
product follows either (orbx_set_nth_pivot), checked by the GPU tests in
tests/test_nth_gpu.py and test_product_nth_pivot_modes below.
"""
import numpy as np
import pytest

from orb_slam_amd import synth
from oracle_lib import RefExtractor, load, ptr


def perm(keys, nth, mode, std_impl=0):
    keys = np.ascontiguousarray(keys, np.float32)
    out = np.zeros(len(keys), np.int32)
    assert load().orbx_ref_nth_element_perm(ptr(keys), len(keys), nth, mode, std_impl, ptr(out)) == 0
    return out


def random_lists(seed=3, count=400):
    r = np.random.default_rng(seed)
    for _ in range(count):
        n = int(r.integers(0, 1500))
        hi = int(r.choice([2, 4, 16, 60, 256]))
        keys = r.integers(0, hi, n).astype(np.float32)
        nth = int(r.integers(0, n + 1)) if n else 0
        yield keys, nth


def test_default_era_is_gcc48():
    """The oracle's default pivot rule is GCC 4.6 .. 4.8's (the product's
    default, include/orbx.h), and RefExtractor uses it unless told."""
    assert load().orbx_ref_get_nth_pivot() == 1
    assert RefExtractor(100).nth_pivot == 1


def test_restatement_equals_std_nth_element():
    """Pivot rule 0 reproduces this image's std::nth_element permutation
    exactly, on random lists with heavy ties and every size class."""
    for keys, nth in random_lists():
        assert np.array_equal(perm(keys, nth, 0), perm(keys, nth, 0, std_impl=1)), (len(keys), nth)


@pytest.mark.parametrize("mode", [0, 1])
def test_both_eras_are_valid_nth_element(mode):
    """Either pivot rule yields an nth_element result: every entry before nth
    is >= keys[nth] >= every entry after it (greater-by-response order)."""
    for keys, nth in random_lists(seed=11, count=200):
        if nth >= len(keys):
            continue
        p = perm(keys, nth, mode)
        assert sorted(p) == list(range(len(keys)))
        k = keys[p]
        assert np.all(k[:nth] >= k[nth]) and np.all(k[nth + 1:] <= k[nth])


def test_eras_differ_on_ties():
    """The two rules are different permutations on tied lists (so the choice
    is observable), and agree when all keys are distinct at the three pivot
    candidates' ranks only by coincidence."""
    differ = sum(not np.array_equal(perm(k, n, 0), perm(k, n, 1)) for k, n in random_lists(seed=5, count=100)
                 if len(k) > 3 and 0 < n < len(k))
    assert differ > 50


def era_difference(frames, nfeatures=1000):
    a, b = RefExtractor(nfeatures, nth_pivot=0), RefExtractor(nfeatures, nth_pivot=1)
    stats = []
    for img in frames:
        ka, da = a(img)
        kb, db = b(img)
        same_order = len(ka) == len(kb) and np.array_equal(ka.view(np.uint8), kb.view(np.uint8))
        sa = {(float(k["x"]), float(k["y"]), int(k["octave"])) for k in ka}
        sb = {(float(k["x"]), float(k["y"]), int(k["octave"])) for k in kb}
        stats.append((same_order, len(sa ^ sb) // 2, len(ka)))
    return stats


def test_era_changes_bench_frames():
    """On the bench's 640x480 sequence the pivot era changes the retained
    keypoint set (tied corners at the cell and level retain boundaries) on
    most frames; the count is what DESIGN.md section 4 reports."""
    stats = era_difference(synth.sequence(640, 480, 4, seed=2000))
    assert sum(not s[0] for s in stats) >= 3
    assert all(s[2] == 1000 for s in stats)


@pytest.mark.gpu
@pytest.mark.parametrize("score_type", [1, 0], ids=["fast", "harris"])
def test_product_nth_pivot_modes(score_type):
    """The device path with the GCC 4.6 .. 4.8 pivot rule equals the oracle
    with the same rule bit for bit (single frames, a 1080p frame whose long
    cell lists take the global-memory replay, and a 48-frame three-part
    batch), and the GCC >= 4.9 rule likewise.  The GCC 4.6 .. 4.8 rule is the
    default of a new context."""
    import orb_slam_amd as ox
    frames = synth.sequence(640, 480, 3, seed=2000)
    ref1 = RefExtractor(1000, score_type=score_type, nth_pivot=1)
    ref0 = RefExtractor(1000, score_type=score_type, nth_pivot=0)
    want = [ref1(f) for f in frames]
    B = 48
    ctx = ox.Context(nfeatures=1000, score_type=score_type, max_w=640, max_h=480, slots=B)
    assert ox.lib().orbx_get_nth_pivot(ctx.handle) == 1   # the default era
    for i, f in enumerate(frames):
        k, d = ctx(f)
        assert np.array_equal(k.view(np.uint8), want[i][0].view(np.uint8)) and np.array_equal(d, want[i][1]), i
    ctx.set_nth_pivot(1)
    for i, f in enumerate(frames):
        k, d = ctx(f)
        assert np.array_equal(k.view(np.uint8), want[i][0].view(np.uint8)) and np.array_equal(d, want[i][1]), i
    ctx.upload(np.stack([frames[i % 3] for i in range(B)]))
    ctx.extract(0, B)
    ctx.sync()
    for s in (0, 1, 2, 16, 17, 31, 32, 47):
        k, d = ctx.features(s)
        rk, rd = want[s % 3]
        assert np.array_equal(k.view(np.uint8), rk.view(np.uint8)) and np.array_equal(d, rd), s
    ctx.set_nth_pivot(0)
    k, d = ctx(frames[0])
    rk, rd = ref0(frames[0])
    assert np.array_equal(k.view(np.uint8), rk.view(np.uint8)) and np.array_equal(d, rd)
    ctx.close()
    big = synth.texture_frame(1920, 1080, 1)
    ctx = ox.Context(nfeatures=2000, score_type=score_type, max_w=1920, max_h=1080, slots=1)
    ctx.set_nth_pivot(1)
    k, d = ctx(big)
    rk, rd = RefExtractor(2000, score_type=score_type, nth_pivot=1)(big)
    assert np.array_equal(k.view(np.uint8), rk.view(np.uint8)) and np.array_equal(d, rd)
    ctx.close()
