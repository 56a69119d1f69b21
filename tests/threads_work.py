"""The workload of the three-thread test (tests/test_threads_gpu.py) and of
bench.py's contention leg: ORB-SLAM's Tracking, LocalMapping and LoopClosing
threads (src/main.cc:122-133), each with its own orbx_ctx, making their
per-frame / per-keyframe calls -- Tracking: orbx_extract ->
orbx_search_by_projection_motion -> orbx_pose_optimization; LocalMapping:
orbx_lba_solve (multi-workgroup) -> orbx_search_for_triangulation;
LoopClosing: orbx_search_by_bow_kf -> orbx_search_by_sim3."""
import ctypes
import threading
import time

import numpy as np

import orb_slam_amd as ox
import proj_data as pd
from bow_data import make_pair
from oracle_lib import RefExtractor, ptr
from orb_slam_amd import synth
from orb_slam_amd import synth_ba as sb
from orb_slam_amd import synth_pose as sp
from test_bow_gpu import run_gpu as bow_gpu
from test_lba_gpu import run_gpu as lba_gpu
from test_pose_gpu import gpu_pose
from test_proj_oracle import ref_sim3, sim3_case

W, H = 640, 480
CAM = np.array([500.0, 500.0, 320.0, 240.0], np.float32)


def _pose_T(tx=-0.008, ty=-0.004, yaw=0.002):
    c, s = np.cos(yaw), np.sin(yaw)
    return np.array([[c, 0, s, tx], [0, 1, 0, ty], [-s, 0, c, 0.0]], np.float32).reshape(-1).copy()


def make_inputs():
    frames = synth.sequence(W, H, 4, seed=91)
    ex = RefExtractor(1000)
    last_k, last_d = ex(frames[0])                       # Tracking's last frame (host features)
    rng = np.random.default_rng(5)
    z = rng.uniform(2.0, 6.0, len(last_k)).astype(np.float32)
    xyz = np.ascontiguousarray(np.stack([(last_k["x"] - CAM[2]) / CAM[0] * z,
                                         (last_k["y"] - CAM[3]) / CAM[1] * z, z], 1).astype(np.float32))
    valid = (rng.random(len(last_k)) < 0.85).astype(np.uint8)
    return dict(
        frames=frames[1:], ref_feats=[ex(f) for f in frames[1:]], last=(last_k, last_d), xyz=xyz, valid=valid,
        T=_pose_T(), pose_frame=sp.make_frame(n_kp=1000, seed=11, outlier_frac=0.1),
        lba=sb.make_problem(n_kf=20, n_points=2000, seed=12, outlier_frac=0.02),
        tri=make_pair(seed=13), bowkf=make_pair(seed=14, n_nodes=20), sim3=sim3_case(15, 0.1))


def _motion(ctx, kc, dc, inp, lib):
    kl, dl = inp["last"]
    C, Lv = ox.frame_view(kc, dc, W, H), ox.frame_view(kl, dl, W, H)
    assigned = np.zeros(len(kc), np.uint8)
    m = np.zeros(len(kc), np.int32)
    n = ctypes.c_int()
    if lib is None:
        assert ox.lib().orbx_search_by_projection_motion(ctx.handle, ctypes.byref(C), ctypes.byref(Lv),
                                                         ox._ptr(inp["xyz"]), ox._ptr(inp["valid"]),
                                                         ox._ptr(assigned), ox._ptr(inp["T"]), ox._ptr(CAM), 15.0, 1,
                                                         ox._ptr(m), ctypes.byref(n)) == 0
    else:
        assert lib.orbx_ref_search_by_projection_motion(ctypes.byref(C), ctypes.byref(Lv), ptr(inp["xyz"]),
                                                        ptr(inp["valid"]), ptr(assigned), ptr(inp["T"]), ptr(CAM),
                                                        15.0, 1, ptr(m), ctypes.byref(n)) == 0
    return m, n.value


def _sim3(ctx, inp, lib=None):
    K1, K2, m1, v1, m2, v2, T1, T2, s12, R12, t12, pr = inp["sim3"][:12]
    if lib is not None:
        return ref_sim3(K1, K2, m1, v1, m2, v2, T1, T2, s12, R12, t12, pr, 7.5)
    gn = np.zeros(K1.n, np.int32)
    gc = ctypes.c_int()
    assert ox.lib().orbx_search_by_sim3(ctx.handle, ctypes.byref(K1), ctypes.byref(K2), ox._ptr(pd.CAM),
                                        ctypes.byref(m1[0]), ox._ptr(v1), ctypes.byref(m2[0]), ox._ptr(v2),
                                        ox._ptr(T1), ox._ptr(T2), float(s12), ox._ptr(R12), ox._ptr(t12), 7.5,
                                        ox._ptr(pr), ox._ptr(gn), ctypes.byref(gc)) == 0
    return gn, gc.value


def tracking(ctx, inp, r):
    f = r % len(inp["frames"])
    t0 = time.perf_counter()
    kps, desc = ctx(inp["frames"][f])
    t1 = time.perf_counter()
    m, n = _motion(ctx, kps, desc, inp, None)
    t2 = time.perf_counter()
    pose = gpu_pose(ctx, [inp["pose_frame"]])[0]
    t3 = time.perf_counter()
    return (kps, desc, m, n, pose), {"extract": t1 - t0, "motion": t2 - t1, "pose": t3 - t2}


def local_mapping(ctx, inp, r):
    t0 = time.perf_counter()
    ba = lba_gpu(ctx, inp["lba"])
    t1 = time.perf_counter()
    tri = bow_gpu(ctx, 2, inp["tri"], 0.6, 1)
    t2 = time.perf_counter()
    return (ba, tri), {"lba": t1 - t0, "triangulation": t2 - t1}


def loop_closing(ctx, inp, r):
    t0 = time.perf_counter()
    bkf = bow_gpu(ctx, 1, inp["bowkf"], 0.75, 1)
    t1 = time.perf_counter()
    s3 = _sim3(ctx, inp)
    t2 = time.perf_counter()
    return (bkf, s3), {"bow_kf": t1 - t0, "sim3": t2 - t1}


def same(a, b):
    """Bit equality of nested outputs (arrays, numbers, ctypes stats)."""
    if isinstance(a, np.ndarray):
        return a.dtype == b.dtype and a.shape == b.shape and a.tobytes() == b.tobytes()
    if isinstance(a, dict):
        return a.keys() == b.keys() and all(same(a[k], b[k]) for k in a)
    if isinstance(a, (tuple, list)):
        return len(a) == len(b) and all(same(x, y) for x, y in zip(a, b))
    if isinstance(a, ctypes.Structure):
        return bytes(a) == bytes(b)
    return a == b


def make_contexts():
    cs = {"tracking": ox.Context(nfeatures=1000, max_w=W, max_h=H, slots=1),
          "local_mapping": ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1),
          "loop_closing": ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)}
    return cs


WORK = {"tracking": tracking, "local_mapping": local_mapping, "loop_closing": loop_closing}


def _medians(times):
    return {k: {c: round(float(np.median([t[c] for t in times[k]])) * 1e3, 4) for c in times[k][0]} for k in times}


def run_threads(contexts, inputs, rounds):
    """The three threads at once, `rounds` rounds each; returns per thread
    the outputs, the per-call times, and any exception text."""
    results = {k: [] for k in WORK}
    times = {k: [] for k in WORK}
    errors = []
    start = threading.Barrier(len(WORK))

    def body(k):
        try:
            start.wait()
            for r in range(rounds):
                o, t = WORK[k](contexts[k], inputs, r)
                results[k].append(o)
                times[k].append(t)
        except BaseException as e:   # reported by the caller
            errors.append((k, repr(e)))

    th = [threading.Thread(target=body, args=(k,)) for k in WORK]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    alive = any(t.is_alive() for t in th)
    return results, times, errors + ([("join", "a thread did not finish")] if alive else [])
