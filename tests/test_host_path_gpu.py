"""The host boundary of the drop-in path on the GPU.

* orbx_extract, the call Frame::Frame makes once per frame
  (src/Frame.cc:59; ORBextractor::operator(), src/ORBextractor.cc:718-779):
  the captured-graph form (orbx_set_launch_mode 1, the default) against the
  stream launches (mode 0) and the oracle, bit-exact, across frame sizes,
  row strides, every configuration switch the graph is keyed on, and the
  error path.
* The host-fed pipeline (orbx_dev_upload_async / orbx_dev_download_async):
  a stream of batches uploaded from page-locked memory and read back into it
  equals the device-resident pipeline's outputs, which equal the oracle's.
"""
import numpy as np
import pytest

import orb_slam_amd as ox
from orb_slam_amd import synth
from oracle_lib import RefExtractor

pytestmark = pytest.mark.gpu


def extract_both(ctx, img, stride=None):
    """(keypoints, descriptors) of one call in each launch mode: the captured
    graph, the stream launches."""
    out = []
    for mode in (1, 0):
        ctx.set_launch_mode(mode)
        out.append(ctx(img) if stride is None else call_strided(ctx, img, stride))
    ctx.set_launch_mode(1)
    return out


def call_strided(ctx, img, stride):
    """orbx_extract on an image embedded in rows of `stride` bytes."""
    import ctypes
    h, w = img.shape
    buf = np.full((h, stride), 0xA5, np.uint8)
    buf[:, :w] = img
    kps = np.zeros(ctx.nfeatures, ox.KEYPOINT)
    desc = np.zeros((ctx.nfeatures, 32), np.uint8)
    n = ctypes.c_int()
    r = ox.lib().orbx_extract(ctx.handle, buf.ctypes.data, w, h, stride, kps.ctypes.data, desc.ctypes.data,
                              ctx.nfeatures, ctypes.byref(n))
    assert r == 0, r
    return kps[:n.value].copy(), desc[:n.value].copy()


def same(a, b):
    return len(a[0]) == len(b[0]) and np.array_equal(a[0].view(np.uint8), b[0].view(np.uint8)) and \
        np.array_equal(a[1], b[1])


@pytest.mark.parametrize("w,h,n,seed", [(640, 480, 1000, 1), (320, 240, 500, 2), (96, 80, 100, 3),
                                        (1920, 1080, 2000, 4)])
def test_graph_call_matches_stream_launches_and_oracle(w, h, n, seed):
    ctx = ox.Context(nfeatures=n, max_w=w, max_h=h, slots=1)
    assert ctx.launch_mode() == 1
    ref = RefExtractor(n)
    for k in range(3):   # first call captures, later calls replay
        img = synth.texture_frame(w, h, seed * 10 + k)
        outs = extract_both(ctx, img)
        r = ref(img)
        assert all(same(o, r) for o in outs), k
    ctx.close()


def test_graph_call_after_size_change_and_with_stride():
    """A smaller frame on the same context re-captures (new geometry), and a
    row stride wider than the image is honoured."""
    ctx = ox.Context(nfeatures=1000, max_w=640, max_h=480, slots=1)
    ref = RefExtractor(1000)
    a = synth.texture_frame(640, 480, 11)
    b = synth.noise_frame(320, 240, 12)
    for img in (a, b, a):
        assert same(ctx(img), ref(img))
    outs = extract_both(ctx, b, stride=352)
    r = ref(b)
    assert all(same(o, r) for o in outs)
    ctx.close()


def test_graph_call_follows_configuration_switches():
    """fp-contract mode and nth_element era changes re-capture: each result
    equals the oracle of the same configuration; launch modes outside 0..1
    are refused."""
    img = synth.noise_frame(640, 480, 21)
    ctx = ox.Context(nfeatures=1000, max_w=640, max_h=480, slots=1)
    assert same(ctx(img), RefExtractor(1000)(img))
    ctx.set_nth_pivot(0)
    assert same(ctx(img), RefExtractor(1000, nth_pivot=0)(img))
    ctx.set_nth_pivot(1)
    ctx.set_fp_contract(1)
    assert same(ctx(img), RefExtractor(1000, variant="contract")(img))
    ctx.set_fp_contract(0)
    for lm in (1, 0, 1):
        ctx.set_launch_mode(lm)
        assert same(ctx(img), RefExtractor(1000)(img)), lm
    for bad in (2, 3, -1):
        assert ox.lib().orbx_set_launch_mode(ctx.handle, bad) == -1
    assert ctx.launch_mode() == 1
    ctx.close()


def test_graph_call_empty_and_capacity():
    """An empty image returns 0 keypoints; a cap below the count is
    ORBX_ERR_CAPACITY with the count reported (both launch modes)."""
    import ctypes
    img = synth.texture_frame(640, 480, 31)
    ctx = ox.Context(nfeatures=1000, max_w=640, max_h=480, slots=1)
    L = ox.lib()
    n = ctypes.c_int(-1)
    assert L.orbx_extract(ctx.handle, None, 0, 0, 0, None, None, 0, ctypes.byref(n)) == 0 and n.value == 0
    for mode in (1, 0):
        ctx.set_launch_mode(mode)
        kps = np.zeros(10, ox.KEYPOINT)
        desc = np.zeros((10, 32), np.uint8)
        r = L.orbx_extract(ctx.handle, img.ctypes.data, 640, 480, 640, kps.ctypes.data, desc.ctypes.data, 10,
                           ctypes.byref(n))
        assert r == -3 and n.value == 1000
    ctx.close()


@pytest.mark.parametrize("mode", ["init", "bf"])
def test_host_fed_pipeline_equals_resident(mode):
    """Batches uploaded asynchronously from page-locked memory (the next
    batch's copy behind this batch's extraction) and read back
    asynchronously equal the device outputs, and those equal the oracle."""
    w, h, B, nf = (640, 480, 48, 1000) if mode == "init" else (320, 240, 16, 500)
    seqs = [synth.sequence(w, h, B, seed=300 + k) for k in range(3)]
    ctx = ox.Context(nfeatures=nf, max_w=w, max_h=h, slots=2 * B)
    ctx.set_async_match(True)
    ctx.upload(seqs[0], first=0)                     # sets the geometry
    src = [ox.HostArray((B, h, w), np.uint8) for _ in seqs]
    for s, q in zip(src, seqs):
        s.array[:] = q
    outs = [dict(kps=ox.HostArray((B * nf,), ox.KEYPOINT), desc=ox.HostArray((B * nf, 32), np.uint8),
                 n=ox.HostArray((B,), np.int32), m12=ox.HostArray((B * nf,), np.int32),
                 nm=ox.HostArray((B,), np.int32)) for _ in seqs]
    ctx.upload_async(src[0].array, first=0)
    for k in range(len(seqs)):
        first = (k % 2) * B
        if k + 1 < len(seqs):
            ctx.upload_async(src[k + 1].array, first=((k + 1) % 2) * B)
        ctx.extract_match(first, B, B, mode=mode, window=100, th_low=50, nnratio=0.9, check_ori=True)
        o = outs[k]
        ctx.download_async(first, B, o["kps"].array, o["desc"].array, o["n"].array, o["m12"].array, o["nm"].array)
    ctx.sync()
    ref = RefExtractor(nf)
    k = len(seqs) - 1
    first, o = (k % 2) * B, outs[k]
    for f in range(B):
        gk, gd = ctx.features(first + f)
        gm, gn = ctx.matches(first + f)
        hk = o["kps"].array[f * nf:f * nf + len(gk)]
        assert int(o["n"].array[f]) == len(gk)
        assert np.array_equal(hk.view(np.uint8), gk.view(np.uint8))
        assert np.array_equal(o["desc"].array[f * nf:f * nf + len(gk)], gd)
        assert int(o["nm"].array[f]) == gn and np.array_equal(o["m12"].array[f * nf:(f + 1) * nf], gm)
    # the earlier batches' host buffers hold their own sequence's results
    for k in range(len(seqs)):
        o = outs[k]
        for f in (0, B - 1):
            rk, rd = ref(seqs[k][f])
            assert int(o["n"].array[f]) == len(rk)
            assert np.array_equal(o["kps"].array[f * nf:f * nf + len(rk)].view(np.uint8), rk.view(np.uint8))
            assert np.array_equal(o["desc"].array[f * nf:f * nf + len(rk)], rd)
    for o in outs:
        for v in o.values():
            v.close()
    for s in src:
        s.close()
    ctx.close()
