"""ctypes binding of the CPU restatement (oracle/liborbx_ref.so).

TEST INFRASTRUCTURE ONLY: the oracle is the parity checker; it is never the
thing measured or shipped.  Built from oracle/ with make when missing (the
prebuilt .so travels to GPU boxes with the snapshot).
"""
import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
ORACLE = ROOT / "oracle"
SO = ORACLE / "liborbx_ref.so"
# the same oracle with src/ORBextractor.cc's own float expressions built as
# GCC builds the reference on an FMA host (oracle/ref_orbsites.cpp)
SO_CONTRACT = ORACLE / "liborbx_ref_contract.so"
KEYPOINT = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

_lib = None
_libs = {}


def build():
    subprocess.run(["make", "-s", "-C", str(ORACLE), "-j8"], check=True)


def load(variant="iso"):
    """The oracle library: variant "iso" (liborbx_ref.so, the parity oracle)
    or "contract" (liborbx_ref_contract.so)."""
    global _lib
    if variant == "iso" and _lib is not None:
        return _lib
    if variant in _libs:
        return _libs[variant]
    path = {"iso": SO, "contract": SO_CONTRACT, "native": ORACLE / "_native" / "liborbx_ref_native.so"}[variant]
    if variant == "iso" and os.environ.get("ORBX_REF_LIBRARY"):   # e.g. the ASan build (test_sanitizers.py)
        path = Path(os.environ["ORBX_REF_LIBRARY"])
    if not path.exists():
        if variant == "native":   # built on the timing host by bench.native_oracle()
            raise FileNotFoundError(path)
        build()
    L = ctypes.CDLL(str(path))
    vp, i, f, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
    ip = ctypes.POINTER(ctypes.c_int)
    sigs = {
        "orbx_ref_extractor_create": ([i, f, i, i, i], vp),
        "orbx_ref_extractor_destroy": ([vp], None),
        "orbx_ref_extract": ([vp, vp, i, i, sz, vp, vp, i, ip], i),
        "orbx_ref_level": ([vp, i, i, vp, i, ip, ip], i),
        "orbx_ref_level_keys": ([vp, i, vp, i, ip], i),
        "orbx_ref_features_per_level": ([vp, vp, i], i),
        "orbx_ref_umax": ([vp, vp, i], i),
        "orbx_ref_scale_factors": ([vp, vp, vp, i], i),
        "orbx_ref_time_extract": ([vp, vp, i, i, i, sz, i], ctypes.c_double),
        "orbx_ref_fast_atan2": ([f, f], f),
        "orbx_ref_cosf": ([f], f),
        "orbx_ref_sinf": ([f], f),
        "orbx_ref_descriptor_distance": ([vp, vp], i),
        "orbx_ref_fast_cell": ([vp, i, i, i, i, vp, i, ip], i),
        "orbx_ref_resize": ([vp, i, i, i, vp, i, i, i], i),
        "orbx_ref_retain_best": ([vp, i, i, vp], i),
        "orbx_ref_search_for_initialization": ([vp, vp, vp, vp, i, f, i, ip], i),
        "orbx_ref_window_search": ([vp, vp, vp, i, i, i, f, i, vp, ip], i),
        "orbx_ref_search_by_projection_pair": ([vp, vp, vp, vp, vp, vp, vp, i, f, vp, ip], i),
        "orbx_ref_search_by_projection_motion": ([vp, vp, vp, vp, vp, vp, vp, f, i, vp, ip], i),
        "orbx_ref_search_by_projection_local": ([vp, i, vp, vp, vp, vp, vp, vp, f, f, vp, ip], i),
        "orbx_ref_hamming_bf": ([vp, i, vp, i, vp, vp, vp], i),
        "orbx_ref_fp_contract": ([], i),
        "orbx_ref_set_nth_pivot": ([i], i),
        "orbx_ref_get_nth_pivot": ([], i),
        "orbx_ref_nth_element_perm": ([vp, i, i, i, i, vp], i),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if variant != "native":   # the native build contracts wherever its host has FMA
        assert L.orbx_ref_fp_contract() == (variant == "contract")
    _libs[variant] = L
    if variant == "iso":
        _lib = L
    return L


def ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class RefExtractor:
    def __init__(self, nfeatures=1000, scale=1.2, nlevels=8, fast_th=20, score_type=1, variant="iso", lib=None,
                 nth_pivot=1):
        self.L = lib if lib is not None else load(variant)
        # retainBest's libstdc++ era (orbx_ref_set_nth_pivot), per call; 1 =
        # GCC 4.6 .. 4.8, the default of the product and the oracle
        self.nth_pivot = nth_pivot
        self.h = self.L.orbx_ref_extractor_create(nfeatures, scale, nlevels, score_type, fast_th)
        assert self.h, "oracle rejected the configuration"
        self.nfeatures = nfeatures
        self.nlevels = nlevels

    def __del__(self):
        try:
            self.L.orbx_ref_extractor_destroy(self.h)
        except Exception:
            pass

    def __call__(self, img):
        img = np.ascontiguousarray(img, np.uint8)
        h, w = img.shape
        kps = np.zeros(self.nfeatures, KEYPOINT)
        desc = np.zeros((self.nfeatures, 32), np.uint8)
        n = ctypes.c_int()
        prev = self.L.orbx_ref_get_nth_pivot()
        assert self.L.orbx_ref_set_nth_pivot(self.nth_pivot) == 0
        try:
            r = self.L.orbx_ref_extract(self.h, ptr(img), w, h, w, ptr(kps), ptr(desc), self.nfeatures,
                                        ctypes.byref(n))
        finally:
            self.L.orbx_ref_set_nth_pivot(prev)
        assert r == 0, r
        return kps[:n.value].copy(), desc[:n.value].copy()

    def level(self, level, blurred=False):
        buf = np.zeros(8 << 20, np.uint8)
        pw, ph = ctypes.c_int(), ctypes.c_int()
        r = self.L.orbx_ref_level(self.h, level, int(blurred), ptr(buf), buf.size, ctypes.byref(pw),
                                  ctypes.byref(ph))
        assert r == 0, r
        return buf[:pw.value * ph.value].reshape(ph.value, pw.value).copy()

    def level_keys(self, level):
        out = np.zeros(self.nfeatures * 4, KEYPOINT)
        n = ctypes.c_int()
        assert self.L.orbx_ref_level_keys(self.h, level, ptr(out), out.size, ctypes.byref(n)) == 0
        return out[:n.value].copy()

    def features_per_level(self):
        out = np.zeros(64, np.int32)
        n = self.L.orbx_ref_features_per_level(self.h, ptr(out), 64)
        return out[:n]

    def umax(self):
        out = np.zeros(32, np.int32)
        n = self.L.orbx_ref_umax(self.h, ptr(out), 32)
        return out[:n]
