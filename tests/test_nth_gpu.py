"""The device introselect replays of k_retain_cells (LDS for lists up to
512 entries, global memory beyond) on adversarial lists, against each other
and against the oracle's retainBest (KeyPointsFilter::retainBest, OpenCV 2.4:
libstdc++ nth_element by response, src/ORBextractor.cc:683, :699): the
first nth entries must be the same entries in the same order."""
import ctypes

import numpy as np
import pytest

import orb_slam_amd as ox
from oracle_lib import load, ptr

pytestmark = pytest.mark.gpu


def lists():
    r = np.random.default_rng(7)
    out = []
    for n in (4, 5, 7, 8, 13, 31, 32, 33, 63, 64, 65, 100, 300, 512):
        out += [("equal", np.full(n, 20)), ("ascending", np.arange(n) % 256), ("descending", (n - np.arange(n)) % 256),
                ("organ", np.minimum(np.arange(n), n - 1 - np.arange(n)) % 256),
                ("ties", r.integers(0, 4, n)), ("scores", r.integers(7, 60, n)),
                ("sawtooth", np.arange(n) % 5)]
    # median-of-three killer style: pushes libstdc++ towards the heap fallback
    for n in (16, 32, 48, 64):
        k = np.zeros(n, np.int64)
        for i in range(n // 2):
            k[2 * i] = i + 1
            k[2 * i + 1] = n // 2 + i + 1
        out.append(("m3killer", k % 256))
    return out


CASES = lists()


@pytest.mark.parametrize("kind,keys", CASES, ids=[f"{k}-{len(v)}" for k, v in CASES])
def test_nth_element_replays(kind, keys):
    L = ox.lib()
    L.orbx_debug_nth.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    R = load()
    n = len(keys)
    entries = ((keys.astype(np.uint32) & 0xFF) << 24 | np.arange(n, dtype=np.uint32)).astype(np.uint32)
    for nth in sorted({1, 2, n // 3, n // 2, n - 1}):
        if not 0 < nth < n:
            continue
        glb = np.zeros(n, np.uint32)
        lds = np.zeros(n, np.uint32)
        assert L.orbx_debug_nth(entries.ctypes.data, n, nth, glb.ctypes.data, lds.ctypes.data) == 0
        assert np.array_equal(glb, lds), (kind, n, nth)
        idx = np.zeros(n, np.int32)
        resp = (entries >> 24).astype(np.float32)
        m = R.orbx_ref_retain_best(ptr(resp), n, nth, ptr(idx))
        assert m >= nth
        assert np.array_equal(lds[:nth] & 0xFFFFFF, idx[:nth]), (kind, n, nth)


@pytest.mark.parametrize("mode", [0, 1], ids=["gcc49", "gcc48"])
@pytest.mark.parametrize("kind,keys", CASES[::3], ids=[f"{k}-{len(v)}" for k, v in CASES[::3]])
def test_nth_element_full_permutation_both_eras(kind, keys, mode):
    """The whole list after the device replay (LDS and global memory) equals
    the oracle's libstdc++ restatement of the same pivot era entry for entry
    (orbx_ref_nth_element_perm), not just the retained prefix."""
    L = ox.lib()
    L.orbx_debug_nth_pivot.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_void_p]
    R = load()
    n = len(keys)
    entries = ((keys.astype(np.uint32) & 0xFF) << 24 | np.arange(n, dtype=np.uint32)).astype(np.uint32)
    resp = (entries >> 24).astype(np.float32)
    for nth in sorted({1, n // 3, n // 2, n - 1}):
        if not 0 < nth < n:
            continue
        glb = np.zeros(n, np.uint32)
        lds = np.zeros(n, np.uint32)
        assert L.orbx_debug_nth_pivot(entries.ctypes.data, n, nth, mode, glb.ctypes.data, lds.ctypes.data) == 0
        perm = np.zeros(n, np.int32)
        assert R.orbx_ref_nth_element_perm(ptr(resp), n, nth, mode, 0, ptr(perm)) == 0
        assert np.array_equal(lds & 0xFFFFFF, perm), (kind, n, nth, mode)
        assert np.array_equal(glb, lds), (kind, n, nth, mode)
