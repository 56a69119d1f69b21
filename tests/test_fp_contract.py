"""FMA contraction of the reference's own float expressions (VERDICT r02,
"unpinned semantics").

The reference is built -O3 -march=native (CMakeLists.txt:12-13); on an FMA
host GCC's default -ffp-contract=fast fuses computeOrbDescriptor's sample
coordinates (src/ORBextractor.cc:165-167) and HarrisResponses' response
(:117-118).  OpenCV 2.4 is a separately built library and is unaffected.
oracle/liborbx_ref_contract.so compiles exactly those expressions
(oracle/ref_orbsites.cpp) the way GCC does for such a build, everything else
shared with the parity oracle; these tests measure what it changes.  The
product reproduces either evaluation (orbx_set_fp_contract), checked
bit-exactly against the matching oracle by the GPU tests at the end.

Measured: FAST_SCORE descriptors differ in one bit
of 400,000 keypoints over 400 640x480 texture / noise frames (seed 386, a
texture frame); keypoints never.  HARRIS_SCORE responses differ on every
frame, which reorders retainBest's ties and changes the keypoint set.
"""
import numpy as np
import pytest

from orb_slam_amd import synth
from oracle_lib import RefExtractor

FLIP_FRAME = dict(w=640, h=480, seed=386)     # the one descriptor flip found (tools: DESIGN.md section 4)


def flip_frame():
    return synth.texture_frame(FLIP_FRAME["w"], FLIP_FRAME["h"], FLIP_FRAME["seed"])


def test_contract_descriptor_flip_is_pinned():
    """On the pinned frame the two evaluations give the same keypoints and
    descriptors that differ in exactly one bit."""
    img = flip_frame()
    ka, da = RefExtractor(1000)(img)
    kb, db = RefExtractor(1000, variant="contract")(img)
    assert np.array_equal(ka.view(np.uint8), kb.view(np.uint8))
    bits = np.unpackbits(da ^ db, axis=1).sum(1)
    assert bits.sum() == 1 and (bits > 0).sum() == 1


@pytest.mark.parametrize("seed", [2000, 2001])
def test_contract_fast_score_sequence_frames_agree(seed):
    """On ordinary frames (the bench's sequences) FAST_SCORE outputs are
    identical under both evaluations."""
    for img in synth.sequence(640, 480, 3, seed=seed):
        ka, da = RefExtractor(1000)(img)
        kb, db = RefExtractor(1000, variant="contract")(img)
        assert np.array_equal(ka.view(np.uint8), kb.view(np.uint8)) and np.array_equal(da, db)


def test_contract_changes_harris_responses():
    """HARRIS_SCORE: the fused response differs from the ISO one on an
    ordinary frame (so HARRIS users must pick the evaluation their reference
    build used)."""
    img = synth.texture_frame(640, 480, 1)
    ka, _ = RefExtractor(1000, score_type=0)(img)
    kb, _ = RefExtractor(1000, score_type=0, variant="contract")(img)
    same = len(ka) == len(kb) and np.array_equal(ka.view(np.uint8), kb.view(np.uint8))
    assert not same


@pytest.mark.gpu
@pytest.mark.parametrize("contract", [0, 1])
@pytest.mark.parametrize("score_type", [1, 0])
def test_product_fp_contract_modes(contract, score_type):
    """The device path in either evaluation equals the oracle built the same
    way, bit for bit, on the pinned flip frame and two sequence frames (FAST
    and HARRIS scores; single-frame and 32-frame batched launches)."""
    import orb_slam_amd as ox
    frames = np.concatenate([flip_frame()[None], synth.sequence(640, 480, 2, seed=2000)])
    B = 32
    batch = np.stack([frames[i % 3] for i in range(B)])
    ctx = ox.Context(nfeatures=1000, score_type=score_type, max_w=640, max_h=480, slots=B)
    ctx.set_fp_contract(contract)
    ref = RefExtractor(1000, score_type=score_type, variant="contract" if contract else "iso")
    want = [ref(f) for f in frames]
    for i, f in enumerate(frames):
        k, d = ctx(f)
        assert np.array_equal(k.view(np.uint8), want[i][0].view(np.uint8)) and np.array_equal(d, want[i][1]), i
    ctx.upload(batch)
    ctx.extract(0, B)
    ctx.sync()
    for s in range(B):
        k, d = ctx.features(s)
        rk, rd = want[s % 3]
        assert np.array_equal(k.view(np.uint8), rk.view(np.uint8)) and np.array_equal(d, rd), s
    ctx.close()
