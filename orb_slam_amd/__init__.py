"""orb_slam_amd -- MI355X-native ORB-SLAM front end and local-BA kernels.

Python view of liborbx (include/orbx.h), used by tests and bench.py.  The
product is the C ABI + HIP kernels in orb_slam_amd/csrc; the production
binding is the C++ adapter in orb_slam_amd/adapters.

There is no CPU fallback: if liborbx.so is missing or no GPU is visible, the
entry points raise.
"""
import ctypes
import os
from pathlib import Path

import numpy as np

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("ORBX_LIBRARY", _PKG / "liborbx.so"))

ORBX_OK = 0
ERRORS = {-1: "ORBX_ERR_ARG", -2: "ORBX_ERR_HIP", -3: "ORBX_ERR_CAPACITY",
          -4: "ORBX_ERR_UNSUPPORTED", -5: "ORBX_ERR_NOMEM", -6: "ORBX_ERR_NOT_POSDEF"}

# cv::KeyPoint / orbx_keypoint (28 bytes)
KEYPOINT = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT.itemsize == 28


class OrbxError(RuntimeError):
    def __init__(self, code, where):
        super().__init__(f"{where}: {ERRORS.get(code, code)}")
        self.code = code


class FrameView(ctypes.Structure):
    _fields_ = [("keys_un", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("n", ctypes.c_int),
                ("min_x", ctypes.c_float), ("max_x", ctypes.c_float),
                ("min_y", ctypes.c_float), ("max_y", ctypes.c_float),
                ("nlevels", ctypes.c_int), ("scale_factor", ctypes.c_float)]


_lib = None


def lib():
    """Load liborbx.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise OrbxError(-2, f"liborbx.so missing at {LIB_PATH}; run python -m orb_slam_amd.build")
        _lib = ctypes.CDLL(str(LIB_PATH))
        _declare(_lib)
    return _lib


def _declare(L):
    vp, i, f, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
    ip = ctypes.POINTER(ctypes.c_int)
    dp = ctypes.POINTER(ctypes.c_double)
    sigs = {
        "orbx_create": ([ctypes.POINTER(vp), i, i, f, i, i, i, i, i, i], i),
        "orbx_destroy": ([vp], None),
        "orbx_get_levels": ([vp], i),
        "orbx_get_scale_factor": ([vp], f),
        "orbx_get_features_per_level": ([vp, vp, i], i),
        "orbx_get_scale_factors": ([vp, vp, i], i),
        "orbx_extract": ([vp, vp, i, i, sz, vp, vp, i, ip], i),
        "orbx_extract_batch": ([vp, i, vp, i, i, sz, vp, vp, i, vp], i),
        "orbx_dev_upload": ([vp, i, i, vp, i, i, sz], i),
        "orbx_dev_extract": ([vp, i, i], i),
        "orbx_dev_match_prev": ([vp, i, i, i, i, f, i], i),
        "orbx_dev_sync": ([vp], i),
        "orbx_dev_match_bf_prev": ([vp, i, i, i, i, f], i),
        "orbx_dev_set_split": ([vp, i], i),
        "orbx_dev_set_async_match": ([vp, i], i),
        "orbx_set_fp_contract": ([vp, i], i),
        "orbx_get_fp_contract": ([vp], i),
        "orbx_set_nth_pivot": ([vp, i], i),
        "orbx_get_nth_pivot": ([vp], i),
        "orbx_dev_extract_match": ([vp, i, i, i, i, i, i, f, i], i),
        "orbx_dev_read_features": ([vp, i, vp, vp, i, ip], i),
        "orbx_dev_read_matches": ([vp, i, vp, i, ip, ip], i),
        "orbx_dev_kernel_time": ([vp, ctypes.c_char_p, dp, dp], i),
        "orbx_dev_kernel_time_enable": ([vp, i], i),
        "orbx_dev_kernel_time_select": ([vp, ctypes.c_char_p], i),
        "orbx_dev_read_level": ([vp, i, i, i, vp, i, ip, ip], i),
        "orbx_descriptor_distance": ([vp, vp], i),
        "orbx_hamming_bf": ([vp, vp, i, vp, i, vp, vp, vp], i),
        "orbx_match_bf": ([vp, vp, i, vp, i, i, f, vp, ip], i),
        "orbx_search_for_initialization": ([vp, vp, vp, vp, vp, i, f, i, ip], i),
        "orbx_window_search": ([vp, vp, vp, vp, i, i, i, f, i, vp, ip], i),
        "orbx_search_by_projection_pair": ([vp, vp, vp, vp, vp, vp, vp, vp, i, f, vp, ip], i),
        "orbx_search_by_projection_motion": ([vp, vp, vp, vp, vp, vp, vp, vp, f, i, vp, ip], i),
        "orbx_search_by_projection_local": ([vp, vp, i, vp, vp, vp, vp, vp, vp, f, f, vp, ip], i),
        "orbx_search_local_map": ([vp, vp], i),
        "orbx_search_local_map_batch": ([vp, i, vp], i),
        "orbx_track_frame": ([vp, vp], i),
        "orbx_lba_solve": ([vp, vp, i, i, vp, vp, vp, vp], i),
        "orbx_lba_solve_batch": ([vp, i, vp, i, i, vp, vp, vp, vp], i),
        "orbx_lba_stage": ([vp, i, vp], i),
        "orbx_lba_run": ([vp, i, i, vp], i),
        "orbx_lba_fetch": ([vp, vp, vp, vp, vp], i),
        "orbx_search_by_bow_frame": ([vp, vp, vp, f, i, vp, ip], i),
        "orbx_search_by_bow_kf": ([vp, vp, vp, f, i, vp, ip], i),
        "orbx_search_for_triangulation": ([vp, vp, vp, vp, vp, i, i, vp, ip], i),
        "orbx_search_for_triangulation_batch": ([vp, vp, i, vp, vp, vp, i, i, vp, vp], i),
        "orbx_search_by_bow_kf_batch": ([vp, vp, i, vp, f, i, vp, vp], i),
        "orbx_fuse_candidates_batch": ([vp, i, vp, vp, vp, vp, i, f, vp, vp], i),
        "orbx_fuse_candidates": ([vp, vp, vp, vp, vp, i, f, vp, vp], i),
        "orbx_dev_fuse_candidates": ([vp, i, vp, vp, vp, vp, vp, i, f, vp, vp], i),
        "orbx_dev_search_by_projection_kf_sim3": ([vp, i, vp, vp, vp, vp, vp, i, vp, i, ip], i),
        "orbx_dev_search_by_projection_frame_kf": ([vp, i, vp, i, vp, vp, vp, vp, vp, f, i, i, vp, i, ip], i),
        "orbx_dev_search_by_sim3": ([vp, i, vp, i, vp, vp, vp, vp, vp, vp, vp, vp, f, vp, vp, f, vp, vp, i, ip], i),
        "orbx_search_by_sim3": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, f, vp, vp, f, vp, vp, ip], i),
        "orbx_distinctive_descriptors": ([vp, i, vp, vp, vp], i),
        "orbx_search_by_projection_kf_sim3": ([vp, vp, vp, vp, vp, vp, i, vp, ip], i),
        "orbx_search_by_projection_frame_kf": ([vp, vp, vp, vp, vp, vp, vp, vp, f, i, i, vp, ip], i),
        "orbx_vocab_create": ([vp, i, i, i, vp, vp, vp, vp, ctypes.POINTER(vp)], i),
        "orbx_vocab_destroy": ([vp], None),
        "orbx_vocab_n_words": ([vp], i),
        "orbx_vocab_transform": ([vp, vp, i, vp, i, vp, vp, vp, vp, vp, ip, vp, vp, vp, ip], i),
        "orbx_dev_compute_bow": ([vp, vp, i, i, i], i),
        "orbx_dev_read_bow": ([vp, i, i, vp, vp, vp, vp, vp, ip, vp, vp, vp, ip], i),
        "orbx_dev_search_by_bow": ([vp, i, i, vp, f, i, vp, i, vp], i),
        "orbx_dev_search_by_bow_kf": ([vp, i, vp, i, vp, vp, f, i, vp, i, vp], i),
        "orbx_dev_search_for_triangulation": ([vp, i, vp, i, vp, vp, vp, vp, i, i, vp, i, vp], i),
        "orbx_undistort_keypoints": ([vp, i, vp, vp, vp, vp], i),
        "orbx_compute_image_bounds": ([i, i, vp, vp, vp], i),
        "orbx_dev_undistort": ([vp, i, i, vp, vp], i),
        "orbx_pose_optimization": ([vp, vp, ip, vp], i),
        "orbx_pose_optimization_batch": ([vp, i, vp, vp, vp], i),
        "orbx_pose_stage": ([vp, i, vp], i),
        "orbx_pose_run": ([vp], i),
        "orbx_pose_fetch": ([vp, vp, vp, vp], i),
        "orbx_version": ([], ctypes.c_char_p),
        "orbx_abi_version": ([], i),
        "orbx_lba_set_workgroups": ([vp, i], i),
        "orbx_lba_get_workgroups": ([vp], i),
        "orbx_lba_last_workgroups": ([vp], i),
        "orbx_debug_lba_split": ([vp, i, i, i, i], i),
        "orbx_pose_set_exact": ([vp, i], i),
        "orbx_pose_get_exact": ([vp], i),
        "orbx_dev_set_image_bounds": ([vp, vp], i),
        "orbx_set_launch_mode": ([vp, i], i),
        "orbx_get_launch_mode": ([vp], i),
        "orbx_host_alloc": ([sz, ctypes.POINTER(vp)], i),
        "orbx_host_free": ([vp], None),
        "orbx_dev_upload_async": ([vp, i, i, vp, i, i, sz], i),
        "orbx_dev_download_async": ([vp, i, i, vp, vp, vp, vp, vp], i),
        "orbx_describe_levels": ([i, f, i, i, i, i, vp, i], i),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _async_array(a, dtype, min_items, name):
    """An asynchronous copy's host array: a HostArray or numpy array of
    `dtype`, C-contiguous (the copy goes through its raw pointer), holding at
    least min_items elements (None: no size requirement); None passes."""
    if a is None:
        return None
    if isinstance(a, HostArray):
        a = a.array
    if not isinstance(a, np.ndarray):
        raise TypeError(f"{name}: expected a numpy array or HostArray, got {type(a).__name__}")
    if a.dtype != np.dtype(dtype):
        raise TypeError(f"{name}: dtype {a.dtype}, expected {np.dtype(dtype)}")
    if not a.flags.c_contiguous:
        raise ValueError(f"{name}: must be C-contiguous")
    if min_items is not None and a.size < min_items:
        raise ValueError(f"{name}: {a.size} elements, the copy writes {min_items}")
    return a


def _check(code, where):
    if code != ORBX_OK:
        raise OrbxError(code, where)


class Context:
    """An orbx_ctx: one device, one HIP stream, `slots` device frame slots.

    Mirrors ORB_SLAM::ORBextractor(nfeatures, scaleFactor, nlevels,
    scoreType, fastTh) (include/ORBextractor.h:37) plus the batched,
    device-resident pipeline.
    """

    def __init__(self, nfeatures=1000, scale_factor=1.2, nlevels=8, score_type=1, fast_th=20,
                 max_w=640, max_h=480, slots=1, device=0):
        self._h = ctypes.c_void_p()
        self.nfeatures = nfeatures
        self.slots = slots
        _check(lib().orbx_create(ctypes.byref(self._h), device, nfeatures, scale_factor, nlevels,
                                 score_type, fast_th, max_w, max_h, slots), "orbx_create")

    def close(self):
        if self._h:
            lib().orbx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- ORBextractor API -------------------------------------------------
    def GetLevels(self):
        return lib().orbx_get_levels(self._h)

    def GetScaleFactor(self):
        return lib().orbx_get_scale_factor(self._h)

    def features_per_level(self):
        out = np.zeros(64, np.int32)
        n = lib().orbx_get_features_per_level(self._h, _ptr(out), 64)
        return out[:n]

    def __call__(self, image, mask=None):
        """ORBextractor::operator()(image, mask, keypoints, descriptors).

        `mask` is accepted and has no effect, as in the reference: it only
        feeds mvMaskPyramid (src/ORBextractor.cc:792-812), whose per-cell
        ROI (:601-603) FAST never reads (:607, :613)."""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape if img.ndim == 2 else (0, 0)
        kps = np.zeros(self.nfeatures, KEYPOINT)
        desc = np.zeros((self.nfeatures, 32), np.uint8)
        n = ctypes.c_int(0)
        _check(lib().orbx_extract(self._h, _ptr(img) if img.size else None, w, h, w, _ptr(kps),
                                  _ptr(desc), self.nfeatures, ctypes.byref(n)), "orbx_extract")
        return kps[:n.value].copy(), desc[:n.value].copy()

    def set_image_bounds(self, bounds=None):
        """orbx_dev_set_image_bounds: (min_x, max_x, min_y, max_y) of the
        slots' undistorted keypoints for the device matchers, None = image."""
        b = None if bounds is None else np.ascontiguousarray(bounds, np.float32)
        _check(lib().orbx_dev_set_image_bounds(self._h, _ptr(b)), "orbx_dev_set_image_bounds")

    def set_launch_mode(self, mode):
        """orbx_extract's launches: 1 one captured hipGraph per call (default),
        0 stream launches (orbx_set_launch_mode)."""
        _check(lib().orbx_set_launch_mode(self._h, int(mode)), "orbx_set_launch_mode")

    def launch_mode(self):
        return lib().orbx_get_launch_mode(self._h)

    # --- device-resident pipeline ------------------------------------------
    def upload(self, frames, first=0):
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        if frames.ndim == 2:
            frames = frames[None]
        cnt, h, w = frames.shape
        _check(lib().orbx_dev_upload(self._h, first, cnt, _ptr(frames), w, h, w), "orbx_dev_upload")

    def upload_async(self, frames, first=0):
        """orbx_dev_upload_async: `frames` (count, h, w) u8, C-contiguous --
        a HostArray (or its .array) for the copy to overlap device work.  The
        memory must stay untouched until the extraction of those slots."""
        frames = _async_array(frames, np.uint8, None, "frames")
        if frames.ndim != 3:
            raise ValueError(f"frames: expected (count, h, w), got shape {frames.shape}")
        cnt, h, w = frames.shape
        _check(lib().orbx_dev_upload_async(self._h, first, cnt, _ptr(frames), w, h, w), "orbx_dev_upload_async")

    def download_async(self, first, count, kps=None, desc=None, n_kps=None, m12=None, n_m=None):
        """orbx_dev_download_async into (preferably page-locked: HostArray)
        arrays: kps count*nfeatures KEYPOINT, desc count*nfeatures*32 u8,
        n_kps count i32, m12 count*nfeatures i32, n_m count i32 (each may be
        None).  The arrays are written when the copy completes (after the
        next call that orders after it, e.g. sync)."""
        nf = self.nfeatures
        kps = _async_array(kps, KEYPOINT, count * nf, "kps")
        desc = _async_array(desc, np.uint8, count * nf * 32, "desc")
        n_kps = _async_array(n_kps, np.int32, count, "n_kps")
        m12 = _async_array(m12, np.int32, count * nf, "m12")
        n_m = _async_array(n_m, np.int32, count, "n_m")
        _check(lib().orbx_dev_download_async(self._h, first, count, _ptr(kps), _ptr(desc), _ptr(n_kps), _ptr(m12),
                                             _ptr(n_m)), "orbx_dev_download_async")

    def extract(self, first, count):
        _check(lib().orbx_dev_extract(self._h, first, count), "orbx_dev_extract")

    def match_prev(self, first, count, seq_len, window=100, nnratio=0.9, check_ori=True):
        _check(lib().orbx_dev_match_prev(self._h, first, count, seq_len, window, nnratio,
                                         int(check_ori)), "orbx_dev_match_prev")

    def extract_match(self, first, count, seq_len, mode="init", window=100, th_low=50, nnratio=0.9,
                      check_ori=True):
        """Extract a batch and match each frame against its predecessor
        (mode "init": SearchForInitialization, "bf": brute force), pipelined."""
        _check(lib().orbx_dev_extract_match(self._h, first, count, seq_len, 1 if mode == "init" else 2, window,
                                            th_low, nnratio, int(check_ori)), "orbx_dev_extract_match")

    def set_split(self, enable):
        """Extraction pipeline parts for a batch (orbx_dev_set_split): 0 one
        stream, 1 the default three parts, 2-4 that many parts on their own
        streams."""
        _check(lib().orbx_dev_set_split(self._h, int(enable)), "orbx_dev_set_split")

    def set_fp_contract(self, enable):
        """Evaluate src/ORBextractor.cc's own float expressions (descriptor
        sample coordinates, Harris response) as a reference build with GCC's
        FMA contraction does (orbx_set_fp_contract)."""
        _check(lib().orbx_set_fp_contract(self._h, int(enable)), "orbx_set_fp_contract")

    def set_nth_pivot(self, mode):
        """retainBest's std::nth_element pivot step as libstdc++ >= 4.9 (0) or
        GCC 4.6 .. 4.8 (1, default: the reference's documented platforms)
        implements it (orbx_set_nth_pivot)."""
        _check(lib().orbx_set_nth_pivot(self._h, int(mode)), "orbx_set_nth_pivot")

    def nth_pivot(self):
        """The retainBest era in effect (orbx_get_nth_pivot)."""
        return lib().orbx_get_nth_pivot(self._h)

    def set_async_match(self, enable):
        """Queue extract_match's matching behind the extraction on an internal
        stream; later extract_match calls on other slots overlap it."""
        _check(lib().orbx_dev_set_async_match(self._h, int(enable)), "orbx_dev_set_async_match")

    def match_bf_prev(self, first, count, seq_len, th_low=50, nnratio=0.9):
        _check(lib().orbx_dev_match_bf_prev(self._h, first, count, seq_len, th_low, nnratio),
               "orbx_dev_match_bf_prev")

    def sync(self):
        _check(lib().orbx_dev_sync(self._h), "orbx_dev_sync")

    def features(self, slot):
        kps = np.zeros(self.nfeatures, KEYPOINT)
        desc = np.zeros((self.nfeatures, 32), np.uint8)
        n = ctypes.c_int(0)
        _check(lib().orbx_dev_read_features(self._h, slot, _ptr(kps), _ptr(desc), self.nfeatures,
                                            ctypes.byref(n)), "orbx_dev_read_features")
        return kps[:n.value].copy(), desc[:n.value].copy()

    def matches(self, slot):
        m = np.zeros(self.nfeatures, np.int32)
        nm, n1 = ctypes.c_int(0), ctypes.c_int(0)
        _check(lib().orbx_dev_read_matches(self._h, slot, _ptr(m), self.nfeatures, ctypes.byref(nm),
                                           ctypes.byref(n1)), "orbx_dev_read_matches")
        return m, nm.value

    def level(self, slot, level, blurred=False, cap=4 << 20):
        buf = np.zeros(cap, np.uint8)
        pw, ph = ctypes.c_int(0), ctypes.c_int(0)
        _check(lib().orbx_dev_read_level(self._h, slot, level, int(blurred), _ptr(buf), cap,
                                         ctypes.byref(pw), ctypes.byref(ph)), "orbx_dev_read_level")
        return buf[:pw.value * ph.value].reshape(ph.value, pw.value).copy()

    def timing(self, enable=True, only=None):
        """Kernel timing with hipEvents around every launch, or only around
        the launches of timer `only`."""
        _check(lib().orbx_dev_kernel_time_select(self._h, only.encode() if only else None), "timing")
        _check(lib().orbx_dev_kernel_time_enable(self._h, int(enable)), "timing")

    def kernel_time(self, name):
        avg, tot = ctypes.c_double(0), ctypes.c_double(0)
        n = lib().orbx_dev_kernel_time(self._h, name.encode(), ctypes.byref(avg), ctypes.byref(tot))
        if n < 0:
            raise OrbxError(n, "orbx_dev_kernel_time")
        return n, avg.value, tot.value

    # --- Optimizer::PoseOptimization --------------------------------------
    def pose_optimization(self, frames):
        """Optimizer::PoseOptimization on a list of orbx_pose_frame structs
        (orb_slam_amd.synth_pose.to_ctypes): updates their Tcw / outlier in
        place, returns (n_inliers, stats)."""
        from .synth_pose import PoseStats
        arr = (type(frames[0]) * len(frames))(*frames)
        n = np.zeros(len(frames), np.int32)
        st = (PoseStats * len(frames))()
        _check(lib().orbx_pose_optimization_batch(self._h, len(frames), arr, _ptr(n), st),
               "orbx_pose_optimization_batch")
        for k in range(len(frames)):
            frames[k].Tcw = arr[k].Tcw
        return n, list(st)

    def pose_stage(self, frames):
        arr = (type(frames[0]) * len(frames))(*frames)
        _check(lib().orbx_pose_stage(self._h, len(frames), arr), "orbx_pose_stage")
        self._pose_staged = arr

    def pose_run(self):
        _check(lib().orbx_pose_run(self._h), "orbx_pose_run")

    def pose_fetch(self):
        from .synth_pose import PoseStats
        arr = self._pose_staged
        n = np.zeros(len(arr), np.int32)
        st = (PoseStats * len(arr))()
        _check(lib().orbx_pose_fetch(self._h, arr, _ptr(n), st), "orbx_pose_fetch")
        return arr, n, list(st)

    # --- DBoW2 on device-resident frames -----------------------------------
    def compute_bow(self, voc, first, count, levelsup=4):
        """Frame::ComputeBoW of extracted slots [first, first+count) on the
        device (orbx_dev_compute_bow); `voc` is a Vocabulary."""
        _check(lib().orbx_dev_compute_bow(self._h, voc.handle, first, count, levelsup), "orbx_dev_compute_bow")

    def read_bow(self, slot):
        """(BowVector, FeatureVector, per-feature (word, weight, node)) of a
        slot as numpy arrays: bow = (words, values); fv = (node ids, CSR
        offsets, feature indices)."""
        n = self.nfeatures
        word, weight, node = np.zeros(n, np.int32), np.zeros(n), np.zeros(n, np.int32)
        bw, bv = np.zeros(n, np.uint32), np.zeros(n)
        fn, fp, ff = np.zeros(n, np.uint32), np.zeros(n + 1, np.int32), np.zeros(n, np.int32)
        nw, nf = ctypes.c_int(), ctypes.c_int()
        _check(lib().orbx_dev_read_bow(self._h, slot, n, _ptr(word), _ptr(weight), _ptr(node), _ptr(bw), _ptr(bv),
                                       ctypes.byref(nw), _ptr(fn), _ptr(fp), _ptr(ff), ctypes.byref(nf)),
               "orbx_dev_read_bow")
        m = int(fp[nf.value])
        return ((bw[:nw.value].copy(), bv[:nw.value].copy()), (fn[:nf.value].copy(), fp[:nf.value + 1].copy(),
                                                               ff[:m].copy()), (word, weight, node))

    def search_by_bow(self, slot, kf_views, nnratio=0.75, check_ori=True):
        """Tracking::Relocalisation's SearchByBoW(pKF, F) loop against the
        frame in `slot` (orbx_dev_search_by_bow): kf_views are orbx_bow_view
        ctypes structures.  Returns (matches per keyframe, counts)."""
        n = len(kf_views)
        outs = [np.zeros(self.nfeatures, np.int32) for _ in range(n)]
        ptrs = (ctypes.c_void_p * max(n, 1))(*[o.ctypes.data for o in outs])
        arr = (type(kf_views[0]) * n)(*kf_views) if n else None
        nm = np.zeros(max(n, 1), np.int32)
        _check(lib().orbx_dev_search_by_bow(self._h, slot, n, arr, nnratio, int(check_ori), ptrs, self.nfeatures,
                                            _ptr(nm)), "orbx_dev_search_by_bow")
        return outs, nm[:n]

    @property
    def handle(self):
        return self._h


class HostArray:
    """Page-locked host memory from orbx_host_alloc viewed as a numpy array
    (freed with the object)."""

    def __init__(self, shape, dtype):
        dtype = np.dtype(dtype)
        n = int(np.prod(shape)) * dtype.itemsize
        self._p = ctypes.c_void_p()
        _check(lib().orbx_host_alloc(max(n, 1), ctypes.byref(self._p)), "orbx_host_alloc")
        buf = (ctypes.c_uint8 * max(n, 1)).from_address(self._p.value)
        self.array = np.frombuffer(buf, np.uint8, count=n).view(dtype).reshape(shape)

    def close(self):
        if self._p:
            self.array = None
            lib().orbx_host_free(self._p)
            self._p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Vocabulary:
    """A DBoW2 vocabulary tree in HBM (orbx_vocab_create): nodes as
    TemplatedVocabulary::loadFromTextFile lists them -- parent id per node
    (node 0 the root), leaf flags, 32-byte descriptors and weights."""

    def __init__(self, ctx, k, L, parent, is_leaf, desc, weight):
        self._keep = [np.ascontiguousarray(parent, np.int32), np.ascontiguousarray(is_leaf, np.uint8),
                      np.ascontiguousarray(desc, np.uint8), np.ascontiguousarray(weight, np.float64)]
        self._h = ctypes.c_void_p()
        _check(lib().orbx_vocab_create(ctx.handle, k, L, len(self._keep[0]), *[_ptr(a) for a in self._keep],
                                       ctypes.byref(self._h)), "orbx_vocab_create")

    @property
    def handle(self):
        return self._h

    def n_words(self):
        return lib().orbx_vocab_n_words(self._h)

    def close(self):
        if self._h:
            lib().orbx_vocab_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def describe_levels(w, h, nfeatures=1000, scale_factor=1.2, nlevels=8, fast_th=20):
    """Per-level host tables of the extractor (no device needed): list of
    dicts {w, h, n_desired, cols, rows, nfeatures_cell, n_cells, n_valid}."""
    out = np.zeros(8 * nlevels, np.int32)
    n = lib().orbx_describe_levels(nfeatures, scale_factor, nlevels, fast_th, w, h, _ptr(out), out.size)
    _check(0 if n > 0 else n, "orbx_describe_levels")
    keys = ["w", "h", "n_desired", "cols", "rows", "nfeatures_cell", "n_cells", "n_valid"]
    return [dict(zip(keys, map(int, out[8 * l:8 * l + 8]))) for l in range(n)]


def frame_view(kps, desc, w, h, nlevels=8, scale_factor=1.2):
    """orbx_frame_view over numpy keypoints/descriptors (Frame without
    distortion: bounds 0..w, 0..h, src/Frame.cc:341-347).  Keep the arrays
    alive while the view is used."""
    v = FrameView()
    v.keys_un = kps.ctypes.data
    v.desc = desc.ctypes.data
    v.n = len(kps)
    v.min_x, v.max_x, v.min_y, v.max_y = 0.0, float(w), 0.0, float(h)
    v.nlevels = nlevels
    v.scale_factor = scale_factor
    return v
