"""Benchmark: frames/sec ORB extract+match (640x480, 1000 kp) on MI355X.

Workloads (BASELINE.json configs):
  c2 (default, the headline metric): synthetic 640x480 mono8 "TUM-style"
     sequences (one per rank, already resident in HBM), 8-level pyramid, 1000
     keypoints.  One step = one batch of B frames: ORB extraction of every
     frame (ORBextractor::operator()) plus SearchForInitialization of every
     frame against its predecessor (window 100, nnratio 0.9, orientation
     check; the sequence is treated as cyclic so every frame is matched).
  c3: 1920x1080, 2000 keypoints, extraction + brute-force Hamming matching of
     every frame against its predecessor (pairs/s; one new pair per frame).
  c5: local BA, 20 keyframes x 2000 map points (5 + 10 LM iterations, two
     outlier passes), a batch of independent problems per step (problems/s);
     inputs cross the host boundary (the reference hands BA its graph from
     host memory), so this rate includes the H2D/D2H copies.
  pose: Optimizer::PoseOptimization: a batch of
     independent 640x480 tracking frames (1000 keypoints, ~70 % with a map
     point, ~10 % gross outliers) staged in HBM once; one step = the full
     four-round robust pose optimisation of every frame from its initial
     pose (frames/s).

Multi-GPU: one process per GPU (torchrun, or `--gpus N` alone: bench.py then
starts the N rank processes itself before any GPU call); each rank owns its
sequence (or problems); the only collective is the end-of-run gather of stats
(RCCL when every rank has its own GPU, gloo when ranks share one).  Weak
scaling: value = units of all ranks / the slowest rank's timed seconds.

Prints ONE JSON line (rank 0) with roofline and cpu_baseline objects.
"""
import argparse
import ctypes
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# A context drives up to six HIP streams (the extraction parts, the match
# stream, the upload stream) besides the null stream.  With HIP's default of
# four hardware queues per process they share queues, and extraction kernels
# queued behind an upload's completion marker wait for the copy: the
# host-inclusive step (tools/host_leg.py, 1024 frames) runs upload + extract
# in 9.97 ms at 4 queues and 5.78 ms at 8 (the copy alone 5.6 ms).  Set before
# anything initialises HIP; rank processes inherit it.
HW_QUEUES = 8
if int(os.environ.get("GPU_MAX_HW_QUEUES") or 4) < HW_QUEUES:
    os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)

import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import dist as odist, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)

WORKLOADS = {
    "c2": dict(w=640, h=480, nfeatures=1000, batch=1024,
               metric="frames/sec ORB extract+match (640x480, 1000 kp)", unit="frames/s",
               desc="640x480 mono8, 8 levels x1.2, 1000 kp: ORB extract + SearchForInitialization vs previous frame"),
    "c3": dict(w=1920, h=1080, nfeatures=2000, batch=128,
               metric="pairs/sec ORB extract + brute-force Hamming match (1920x1080, 2000 kp)", unit="pairs/s",
               desc="1920x1080 mono8, 8 levels x1.2, 2000 kp: ORB extract + brute-force Hamming vs previous frame"),
    "c5": dict(batch=256, metric="local BA problems/sec (20 KF x 2000 MP, 5+10 LM iterations)", unit="problems/s",
               desc="Optimizer::LocalBundleAdjustment core: 20 keyframes (+2 fixed) x 2000 map points, "
                    "Huber, Schur + LLT, 5+10 LM iterations, two outlier passes"),
    "pose": dict(batch=8192, metric="frames/sec Optimizer::PoseOptimization (1000 kp, ~700 map points)",
                 unit="frames/s",
                 desc="Optimizer::PoseOptimization: 1000 keypoints, ~700 map-point edges, ~10 % outliers, "
                      "Huber, 4 robust rounds (10/10/7/5 LM iterations), Eigen-LDLT 6x6 trials"),
}

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (AMD spec: 256 CU x 128 FLOP/clk x 2.4 GHz)


def level_sizes(w, h, nlevels=8, scale=1.2):
    sizes = []
    invf = np.float32(1.0 / np.float64(np.float32(scale)))
    s = np.float32(1.0)
    for l in range(nlevels):
        sizes.append((int(np.rint(np.float32(w) * s)), int(np.rint(np.float32(h) * s))))
        s = np.float32(s * invf)
    return sizes


def algorithmic_bytes(w, h, nfeatures, match="init"):
    """Per-frame algorithmic bytes per stage: each
    stage's compulsory HBM reads + writes of its inputs/outputs."""
    sz = level_sizes(w, h)
    px = [a * b for a, b in sz]
    return {
        "pyr0": px[0] + px[0],                               # read image, write level 0
        "resize": sum(px[l - 1] + px[l] for l in range(1, 8)),
        "fast": sum(px),                                     # one read of every level
        "blur": 2 * sum(px),                                 # read + write
        "describe": nfeatures * (512 + 700 + 60),            # samples, IC patch, outputs
        "retain": 0,
        "match": (2 * nfeatures * 32 + nfeatures * 4) if match == "bf" else 0,
    }


def survey_frame_bytes(w, h, nfeatures):
    """SURVEY.md 8(d) B_frame: sum_{l>=1}(px_l + px_{l-1}) pyramid write + read,
    sum_l px_l FAST read, 2 sum_l px_l blur read + write, N_kp (32 + 28)
    outputs (4.48 MB at 640x480 / 1000 kp)."""
    px = [a * b for a, b in level_sizes(w, h)]
    return sum(px[l] + px[l - 1] for l in range(1, len(px))) + 3 * sum(px) + nfeatures * (32 + 28)


def lba_bytes(n_kf, n_pts, n_edges):
    """Algorithmic bytes of one LM iteration."""
    return n_edges * (2 * 8 + 4 + 8) + n_edges * 144 + n_kf * 7 * 8 + n_pts * 3 * 8


def native_oracle():
    """The timed CPU baseline's library: the oracle built on THIS host with
    the reference's own flags, -O3 -march=native (CMakeLists.txt:12-13;
    SURVEY.md 8(d)), by `make -C oracle native`, rebuilt when the host CPU
    differs from the one it was built for.  Falls back to the portable
    x86-64-v3 parity build (oracle/liborbx_ref.so) if that fails.
    Returns (ctypes library, description)."""
    import hashlib
    import subprocess
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    try:
        cpu = Path("/proc/cpuinfo").read_text()
        sig = hashlib.sha256("".join(l for l in cpu.splitlines(True)[:40]
                                     if l.startswith(("model name", "flags"))).encode()).hexdigest()[:16]
    except OSError:
        sig = "unknown"
    nat = ROOT / "oracle" / "_native"
    so = nat / "liborbx_ref_native.so"
    stamp = nat / "HOST"
    try:
        if nat.exists() and (not stamp.exists() or stamp.read_text() != sig):   # built for another CPU
            subprocess.run(["rm", "-rf", str(nat)], check=True)
        # incremental: also picks up oracle sources newer than the objects
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "-j16", "native"], check=True,
                       capture_output=True, timeout=240)
        stamp.write_text(sig)
        return oracle_lib.load("native"), "oracle/_native/liborbx_ref_native.so (g++ -O3 -march=native, built on this host)"
    except Exception as e:   # noqa: BLE001 -- a baseline, not the product: say what was timed
        return oracle_lib.load(), f"oracle/liborbx_ref.so (g++ -O3 -march=x86-64-v3; native build failed: {e!r:.80})"


def percentile_summary(times_s, unit_name):
    t = np.asarray(times_s)
    med, p90 = float(np.median(t)), float(np.percentile(t, 90))
    return {"value": round(1.0 / med, 3), "median_ms": round(1e3 * med, 4), "p90_ms": round(1e3 * p90, 4),
            "mean_rate": round(len(t) / float(t.sum()), 3), "timed_units": len(t), "rate_from": f"1 / median {unit_name} time"}


# SURVEY.md 8(d) protocol: warm-up units, then the median (and p90) of the
# per-unit times of `timed` units.  C3's 1080p frames take ~65 ms each, so
# its sample is shorter (stated in the line).
CPU_PROTOCOL = {"c2": (50, 500), "c3": (10, 150), "c5": (50, 500), "pose": (50, 500)}


def cpu_baseline_frames(frames, nfeatures, protocol, bf=False, L=None, lib_desc=""):
    """Oracle on one host core, per frame: extract + match against the
    previous frame of the same sequence (the bench's unit)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    if L is None:
        L, lib_desc = native_oracle()
    ex = oracle_lib.RefExtractor(nfeatures, lib=L)
    h, w = frames.shape[1:]
    warm, timed_n = protocol
    times = []
    prev = None
    for n in range(warm + timed_n):
        t0 = time.perf_counter()
        k, d = ex(frames[n % len(frames)])
        if prev is not None:
            if bf:
                bi, b1, b2 = (np.zeros(len(prev[1]), np.int32) for _ in range(3))
                L.orbx_ref_hamming_bf(oracle_lib.ptr(prev[1]), len(prev[1]), oracle_lib.ptr(d), len(d),
                                      oracle_lib.ptr(bi), oracle_lib.ptr(b1), oracle_lib.ptr(b2))
            else:
                F1 = ox.frame_view(prev[0], prev[1], w, h)
                F2 = ox.frame_view(k, d, w, h)
                pm = np.stack([prev[0]["x"], prev[0]["y"]], 1).astype(np.float32).copy()
                m = np.zeros(len(prev[0]), np.int32)
                nm = ctypes.c_int()
                L.orbx_ref_search_for_initialization(ctypes.byref(F1), ctypes.byref(F2), oracle_lib.ptr(pm),
                                                     oracle_lib.ptr(m), 100, 0.9, 1, ctypes.byref(nm))
        dt = time.perf_counter() - t0
        if n >= warm:
            times.append(dt)
        prev = (k, d)
    what = "brute-force Hamming" if bf else "SearchForInitialization"
    out = {"unit": "pairs/s" if bf else "frames/s", "cores": 1, "kind": "port"}
    out.update(percentile_summary(times, "frame"))
    out["sample"] = (f"{warm} warm-up + {timed_n} timed frames of the same synthetic sequence ({w}x{h}), extract + "
                     f"{what} vs the previous frame, 1 thread; {lib_desc}")
    return out


def cpu_threads():
    """Host threads for the all-cores CPU baseline: the box's CPU share
    (OMP_NUM_THREADS is set to it on the GPU box), else the visible cores."""
    for key in ("ORBX_CPU_THREADS", "OMP_NUM_THREADS"):
        if os.environ.get(key, "").isdigit() and int(os.environ[key]) > 0:
            return min(int(os.environ[key]), 64)
    return min(os.cpu_count() or 1, 64)


def run_threads(n_threads, budget_s, worker):
    """worker(t, deadline) -> units done; the oracle's C calls release the
    GIL, so the threads run on separate cores.  Returns (units, seconds)."""
    import threading
    counts = [0] * n_threads
    t0 = time.perf_counter()
    deadline = t0 + budget_s

    def run(t):
        counts[t] = worker(t, deadline)

    ths = [threading.Thread(target=run, args=(t,)) for t in range(n_threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    return sum(counts), time.perf_counter() - t0


def cpu_all_cores_frames(frames, nfeatures, budget_s, bf=False, L=None, lib_desc=""):
    """the oracle on every host core, one frame stream per
    thread (extract + match against that stream's previous frame)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    if L is None:
        L, lib_desc = native_oracle()
    h, w = frames.shape[1:]
    T = cpu_threads()

    def worker(t, deadline):
        ex = oracle_lib.RefExtractor(nfeatures, lib=L)
        n, prev = 0, None
        while time.perf_counter() < deadline:
            k, d = ex(frames[(t + n * T) % len(frames)])
            if prev is not None:
                if bf:
                    bi, b1, b2 = (np.zeros(len(prev[1]), np.int32) for _ in range(3))
                    L.orbx_ref_hamming_bf(oracle_lib.ptr(prev[1]), len(prev[1]), oracle_lib.ptr(d), len(d),
                                          oracle_lib.ptr(bi), oracle_lib.ptr(b1), oracle_lib.ptr(b2))
                else:
                    F1 = ox.frame_view(prev[0], prev[1], w, h)
                    F2 = ox.frame_view(k, d, w, h)
                    pm = np.stack([prev[0]["x"], prev[0]["y"]], 1).astype(np.float32).copy()
                    m = np.zeros(len(prev[0]), np.int32)
                    nm = ctypes.c_int()
                    L.orbx_ref_search_for_initialization(ctypes.byref(F1), ctypes.byref(F2), oracle_lib.ptr(pm),
                                                         oracle_lib.ptr(m), 100, 0.9, 1, ctypes.byref(nm))
            prev = (k, d)
            n += 1
        return n

    n, dt = run_threads(T, budget_s, worker)
    return {"value": round(n / dt, 3), "unit": "pairs/s" if bf else "frames/s", "cores": T, "kind": "port",
            "sample": f"{n} frames ({w}x{h}) on {T} threads, one frame stream each, {dt:.1f} s; {lib_desc}"}


def cpu_baseline_lba(probs, protocol, L=None, lib_desc=""):
    sys.path.insert(0, str(ROOT / "tests"))
    from orb_slam_amd import synth_ba as sb
    if L is None:
        L, lib_desc = native_oracle()
    L.orbx_ref_lba.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p]
    warm, timed_n = protocol
    times = []
    for n in range(warm + timed_n):
        p, arrs = sb.to_ctypes(probs[n % len(probs)])
        es = np.zeros(p.n_edges, np.uint8)
        pb = np.zeros(p.n_points, np.uint8)
        st = sb.BAStats()
        t0 = time.perf_counter()
        L.orbx_ref_lba(ctypes.byref(p), 5, 10, es.ctypes.data, pb.ctypes.data, ctypes.byref(st))
        if n >= warm:
            times.append(time.perf_counter() - t0)
    out = {"unit": "problems/s", "cores": 1, "kind": "port"}
    out.update(percentile_summary(times, "problem"))
    out["sample"] = (f"{warm} warm-up + {timed_n} timed problems (20 KF x 2000 MP), oracle LBA (dense LLT in place "
                     f"of CHOLMOD), 1 thread; {lib_desc}")
    return out


def lba_flops(prob, stats):
    """FP64 flops of one local-BA solve by SURVEY.md 8(d)'s per-iteration
    formula: E (~150 linearize + ~250 accumulate) per LM iteration, and per
    trial the Schur complement sum_points k^2 216 (k = the point's edges to
    free poses) plus the (6P)^3 / 3 factorisation; both optimize() passes
    with their iteration / trial counts (the second pass on the edge set
    left after the first outlier pass, approximated by the full set)."""
    free = prob["pose_fixed"] == 0
    ep = np.asarray(prob["edge_pose"])
    k = np.bincount(np.asarray(prob["edge_point"])[free[ep]], minlength=len(prob["point_id"]))
    E = len(ep)
    per_iter = E * 400.0
    per_trial = float((k.astype(np.float64) ** 2).sum()) * 216.0 + (6.0 * free.sum()) ** 3 / 3.0
    return sum(stats.iterations[p] * per_iter + stats.levenberg_trials[p] * per_trial for p in range(2))


def pose_flops(stats, n_edges):
    """FP64 flops of one PoseOptimization from its LM statistics: ~215 per
    edge per fused error+Jacobian+H pass (one per LM iteration), ~55 per edge
    per trial error pass and per classification (counted from the kernel's
    arithmetic; orb_slam_amd/csrc/orbx_pose.hip)."""
    f = 0.0
    active = n_edges
    for r in range(stats.rounds):
        f += stats.iterations[r] * 215.0 * active + stats.levenberg_trials[r] * 55.0 * active + 55.0 * n_edges
        active = n_edges - stats.n_bad[r]
    return f


def cpu_all_cores_lba(probs, budget_s, L=None, lib_desc=""):
    sys.path.insert(0, str(ROOT / "tests"))
    from orb_slam_amd import synth_ba as sb
    if L is None:
        L, lib_desc = native_oracle()
    L.orbx_ref_lba.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p]
    T = cpu_threads()

    def worker(t, deadline):
        n = 0
        while time.perf_counter() < deadline:
            p, arrs = sb.to_ctypes(probs[(t + n * T) % len(probs)])
            es = np.zeros(p.n_edges, np.uint8)
            pb = np.zeros(p.n_points, np.uint8)
            L.orbx_ref_lba(ctypes.byref(p), 5, 10, es.ctypes.data, pb.ctypes.data, ctypes.byref(sb.BAStats()))
            n += 1
        return n

    n, dt = run_threads(T, budget_s, worker)
    return {"value": round(n / dt, 4), "unit": "problems/s", "cores": T, "kind": "port",
            "sample": f"{n} problems on {T} threads, {dt:.1f} s; {lib_desc}"}


def cpu_all_cores_pose(frames, budget_s, L=None, lib_desc=""):
    sys.path.insert(0, str(ROOT / "tests"))
    from orb_slam_amd import synth_pose as sp
    if L is None:
        L, lib_desc = native_oracle()
    L.orbx_ref_pose_optimization.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    structs = [sp.to_ctypes(fr) for fr in frames]
    T = cpu_threads()

    def worker(t, deadline):
        n = 0
        while time.perf_counter() < deadline:
            p, arrs = structs[(t + n * T) % len(structs)]
            q = sp.PoseFrame.from_buffer_copy(p)
            L.orbx_ref_pose_optimization(ctypes.byref(q), None, None)
            n += 1
        return n

    n, dt = run_threads(T, budget_s, worker)
    return {"value": round(n / dt, 3), "unit": "frames/s", "cores": T, "kind": "port",
            "sample": f"{n} frames on {T} threads, {dt:.1f} s; {lib_desc}"}


def cpu_baseline_pose(frames, protocol, L=None, lib_desc=""):
    sys.path.insert(0, str(ROOT / "tests"))
    from orb_slam_amd import synth_pose as sp
    if L is None:
        L, lib_desc = native_oracle()
    L.orbx_ref_pose_optimization.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    structs = [sp.to_ctypes(fr) for fr in frames]
    warm, timed_n = protocol
    times = []
    for n in range(warm + timed_n):
        p, arrs = structs[n % len(structs)]
        q = sp.PoseFrame.from_buffer_copy(p)          # fresh initial pose each time
        t0 = time.perf_counter()
        L.orbx_ref_pose_optimization(ctypes.byref(q), None, None)
        if n >= warm:
            times.append(time.perf_counter() - t0)
    out = {"unit": "frames/s", "cores": 1, "kind": "port"}
    out.update(percentile_summary(times, "frame"))
    out["sample"] = (f"{warm} warm-up + {timed_n} timed frames of the same synthetic set, oracle PoseOptimization "
                     f"(Eigen-LDLT restatement), 1 thread; {lib_desc}")
    return out


def parity_pose(uniq, arr, n_inl, sample=(0, 1, 2, 3, 127, 255)):
    """The last timed step's Tcw of a few frames against the oracle's
    PoseOptimization from the same initial pose (1e-5, the north_star pose
    tolerance; identical inlier counts)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    from orb_slam_amd import synth_pose as sp
    L = oracle_lib.load()
    L.orbx_ref_pose_optimization.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.orbx_ref_pose_optimization.restype = ctypes.c_int
    worst, bad = 0.0, []
    for i in sample:
        if i >= len(uniq):
            continue
        p, arrs = sp.to_ctypes(uniq[i])
        ni = ctypes.c_int()
        r = L.orbx_ref_pose_optimization(ctypes.byref(p), ctypes.byref(ni), None)
        d = float(np.abs(np.ctypeslib.as_array(arr[i].Tcw) - np.ctypeslib.as_array(p.Tcw)).max())
        worst = max(worst, d)
        if r != 0 or d > 1e-5 or ni.value != int(n_inl[i]):
            bad.append(i)
    return {"within_1e-5": not bad, "max_abs_tcw_diff": worst, "frames": list(sample), "mismatched": bad,
            "oracle": "oracle/liborbx_ref.so"}


def run_pose(args, wl, rank, local, world, dist):
    from orb_slam_amd import synth_pose as sp
    P = args.batch or wl["batch"]
    uniq = [sp.make_frame(n_kp=1000, seed=odist.shard_seed(7000, rank) * 1000 + i) for i in range(min(P, 256))]
    frames = [uniq[i % len(uniq)] for i in range(P)]
    ctx = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1, device=args.device)
    if args.pose_fast_sums and ox.lib().orbx_pose_set_exact(ctx.handle, 0) != 0:
        raise RuntimeError("orbx_pose_set_exact failed")
    keep = [sp.to_ctypes(fr) for fr in frames]
    ctx.pose_stage([k[0] for k in keep])
    n_edges = int(np.mean([fr["has_mp"].sum() for fr in uniq]))

    def step():
        ctx.pose_run()

    for _ in range(args.warmup):
        step()
    elapsed, kernels = timed(args, ctx, step, dist, ["pose"])
    kernels = {"timed": None, "serial": kernels, "serial_steps": args.steps}   # one launch per step
    arr, n_inl, st = ctx.pose_fetch()
    stats = np.array([elapsed, P * args.steps, int(n_inl[0]), st[0].rounds], dtype=np.float64)
    allst = odist.gather_stats(stats, dist, device=args.gather_device)   # before rank 0's CPU legs
    ab = {"pose": n_edges * 25 + 80 + 160}
    units_per_step = {"pose": P}
    flops = float(np.mean([pose_flops(st[i], int(frames[i]["has_mp"].sum())) for i in range(len(uniq))]))
    cpu = None
    check = {"inliers_frame0": int(n_inl[0]), "edges_frame0": int(frames[0]["has_mp"].sum()),
             "rounds_frame0": int(st[0].rounds), "lm_iterations_frame0": list(st[0].iterations),
             "fp64_flops_per_frame": round(flops)}
    if rank == 0 and not args.no_cpu_baseline:
        check["parity_last_step"] = parity_pose(uniq, arr, n_inl)
        L, desc = native_oracle()
        cpu = cpu_baseline_pose(uniq, CPU_PROTOCOL["pose"], L=L, lib_desc=desc)
        cpu["all_cores"] = cpu_all_cores_pose(uniq, max(3.0, args.cpu_budget / 2), L=L, lib_desc=desc)
    cfg = {"workload": wl["desc"], "frames_per_step_per_gpu": P, "keypoints": 1000, "map_point_edges": n_edges,
           "parallelism": f"dp{world} (independent frames per GPU)",
           "sums": "lane-strided + fixed DPP tree (opt-in fast sums, orbx_pose_set_exact(ctx, 0))"
                   if args.pose_fast_sums else "sequential in g2o's edge order (default)",
           "boundary": "frames staged in HBM before the timed region (orbx_pose_stage); results fetched after"}
    ctx.close()
    return allst, kernels, ab, units_per_step, cpu, check, cfg


# Single-call legs (VERDICT r04 "Next" #1): the reference calls the hot path
# one unit at a time, synchronously -- the extractor once per frame
# (src/Frame.cc:59 from src/Tracking.cc:206), SearchForInitialization per
# initialisation attempt (src/Tracking.cc:361), PoseOptimization 2-4 times per
# frame (src/Tracking.cc:533,556,593,627), LocalBundleAdjustment once per
# keyframe (src/LocalMapping.cc:83).  Each leg times the same C-ABI call the
# C++ adapter makes (orb_slam_amd/adapters/orbx_adapters.hpp), host arrays in
# and out, one call at a time: 50 warm-up calls, then the median (and p90) of
# 500; the oracle's single-thread call on the same inputs beside it.
SINGLE_PROTOCOL = (50, 500)


def time_calls(fn, n_items, protocol, reset=None):
    """Per-call wall times of fn(i) (reset(i) runs before each call, untimed)."""
    warm, timed_n = protocol
    times = []
    for k in range(warm + timed_n):
        if reset is not None:
            reset(k % n_items)
        t0 = time.perf_counter()
        fn(k % n_items)
        dt = time.perf_counter() - t0
        if k >= warm:
            times.append(dt)
    t = np.asarray(times)
    return {"median_ms": round(1e3 * float(np.median(t)), 4), "p90_ms": round(1e3 * float(np.percentile(t, 90)), 4),
            "calls": len(t)}


def single_call_legs(args, frames, nf, w, h):
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    from orb_slam_amd import synth_ba as sb, synth_pose as sp
    L = ox.lib()
    R, rdesc = native_oracle()
    proto = SINGLE_PROTOCOL
    out = {"protocol": f"{proto[0]} warm-up calls, then the median / p90 of {proto[1]}; one call at a time, "
                       "host arrays in and out (the adapter's C-ABI call); cpu = the oracle on one core "
                       f"({rdesc})"}

    def check_rc(r, where):
        if r != 0:
            raise ox.OrbxError(r, where)

    # --- ORBextractor::operator() on one 640x480 frame --------------------
    imgs = [np.ascontiguousarray(f) for f in frames[:64]]
    ctx1 = ox.Context(nfeatures=nf, max_w=w, max_h=h, slots=1, device=args.device)
    kps = np.zeros(nf, ox.KEYPOINT)
    desc = np.zeros((nf, 32), np.uint8)
    n = ctypes.c_int()

    def ext(i):
        check_rc(L.orbx_extract(ctx1.handle, imgs[i].ctypes.data, w, h, w, kps.ctypes.data, desc.ctypes.data, nf,
                                ctypes.byref(n)), "orbx_extract")

    ex = {}
    for mode, name in ((1, "graph"), (0, "stream_launches")):
        ctx1.set_launch_mode(mode)
        ex[name] = time_calls(ext, len(imgs), proto)
    ctx1.set_launch_mode(1)
    rex = oracle_lib.RefExtractor(nf, lib=R, nth_pivot=ctx1.nth_pivot())          # timed (reference flags)
    rpar = oracle_lib.RefExtractor(nf, nth_pivot=ctx1.nth_pivot())                # parity oracle
    bad = []
    for i in (0, 1, 63):                      # graph-path outputs against the oracle
        ext(i)
        rk, rd = rpar(imgs[i])
        if not (n.value == len(rk) and np.array_equal(kps[:n.value].view(np.uint8), rk.view(np.uint8))
                and np.array_equal(desc[:n.value], rd)):
            bad.append(i)
    ex["cpu"] = time_calls(lambda i: rex(imgs[i]), len(imgs), proto)
    ex["speedup_vs_cpu"] = round(ex["cpu"]["median_ms"] / ex["graph"]["median_ms"], 2)
    ex["graph_vs_stream_launches"] = round(ex["stream_launches"]["median_ms"] / ex["graph"]["median_ms"], 2)
    ex["bit_exact"] = not bad
    ex["call"] = (f"orbx_extract: one {w}x{h} mono8 host image in, {nf}-keypoint records + descriptors out "
                  "(ORBextractor::operator(), src/ORBextractor.cc:718-779)")
    out["extract"] = ex

    # --- SearchForInitialization on consecutive frames (host views) --------
    feats = [rex(imgs[i]) for i in range(8)]
    views = [(ox.frame_view(k, d, w, h), k, d) for k, d in feats]
    m12 = np.zeros(nf, np.int32)
    pm = np.zeros((nf, 2), np.float32)
    nm = ctypes.c_int()

    def prev_reset(i):
        k = views[i][1]
        pm[:len(k)] = np.stack([k["x"], k["y"]], 1)

    def sfi(i, lib_call):
        F1, F2 = views[i][0], views[(i + 1) % len(views)][0]
        lib_call(F1, F2)

    def gpu_sfi(F1, F2):
        check_rc(L.orbx_search_for_initialization(ctx1.handle, ctypes.byref(F1), ctypes.byref(F2), pm.ctypes.data,
                                                  m12.ctypes.data, 100, 0.9, 1, ctypes.byref(nm)),
                 "orbx_search_for_initialization")

    def cpu_sfi(F1, F2):
        R.orbx_ref_search_for_initialization(ctypes.byref(F1), ctypes.byref(F2), pm.ctypes.data, m12.ctypes.data,
                                             100, 0.9, 1, ctypes.byref(nm))

    mt = {"gpu": time_calls(lambda i: sfi(i, gpu_sfi), len(views), proto, reset=prev_reset),
          "cpu": time_calls(lambda i: sfi(i, cpu_sfi), len(views), proto, reset=prev_reset)}
    mt["speedup_vs_cpu"] = round(mt["cpu"]["median_ms"] / mt["gpu"]["median_ms"], 2)
    mt["call"] = ("orbx_search_for_initialization: two host frame views (1000 keypoints each), window 100, nnratio "
                  "0.9, orientation check (ORBmatcher::SearchForInitialization, src/ORBmatcher.cc:598-713)")
    out["search_for_initialization"] = mt

    # --- Tracking's per-frame window / projection searches (host views) ------
    # TrackWithMotionModel's SearchByProjection (src/Tracking.cc:584, th 15),
    # TrackPreviousFrame's WindowSearch (:510, window 200) and pair search
    # (:544, window 15), SearchReferencePointsInFrustum's local-map search
    # (:745-750, th 1): the two-phase kernels (k_area_lists + k_area_replay)
    cam = np.array([500.0, 500.0, 320.0, 240.0], np.float32)
    (kl, dl), (kc, dc) = feats[0], feats[1]
    Lv, Cv = views[0][0], views[1][0]
    rng = np.random.default_rng(31)
    z = rng.uniform(2.0, 6.0, len(kl)).astype(np.float32)
    xyz = np.ascontiguousarray(np.stack([(kl["x"] - cam[2]) / cam[0] * z, (kl["y"] - cam[3]) / cam[1] * z, z],
                                        1).astype(np.float32))
    valid = (rng.random(len(kl)) < 0.85).astype(np.uint8)
    asg = np.zeros(len(kc), np.uint8)
    c_, s_ = np.cos(0.002), np.sin(0.002)
    T = np.array([[c_, 0, s_, -0.008], [0, 1, 0, -0.004], [-s_, 0, c_, 0.0]], np.float32).reshape(-1).copy()
    proj = np.ascontiguousarray(np.stack([kl["x"] + 2.0, kl["y"] + 1.0], 1).astype(np.float32))
    pred = np.ascontiguousarray(kl["octave"].astype(np.int32))
    vcos = rng.uniform(0.99, 1.0, len(kl)).astype(np.float32)
    mpd = np.ascontiguousarray(dl)
    m_out = np.zeros(nf, np.int32)
    P = oracle_lib.load()   # the parity oracle (R, the native build, is the timed one)
    searches = {
        "motion_th15": (
            lambda lib_: lib_.orbx_ref_search_by_projection_motion(ctypes.byref(Cv), ctypes.byref(Lv), xyz.ctypes.data,
                                                                   valid.ctypes.data, asg.ctypes.data, T.ctypes.data,
                                                                   cam.ctypes.data, ctypes.c_float(15.0), 1,
                                                                   m_out.ctypes.data, ctypes.byref(nm)),
            lambda: L.orbx_search_by_projection_motion(ctx1.handle, ctypes.byref(Cv), ctypes.byref(Lv), xyz.ctypes.data,
                                                       valid.ctypes.data, asg.ctypes.data, T.ctypes.data,
                                                       cam.ctypes.data, 15.0, 1, m_out.ctypes.data, ctypes.byref(nm)),
            "SearchByProjection(Frame&, const Frame&, th 15) (src/ORBmatcher.cc:1507-1620)"),
        "window_200": (
            lambda lib_: lib_.orbx_ref_window_search(ctypes.byref(Lv), ctypes.byref(Cv), valid.ctypes.data, 200, 0, -1,
                                                     ctypes.c_float(0.9), 1, m_out.ctypes.data, ctypes.byref(nm)),
            lambda: L.orbx_window_search(ctx1.handle, ctypes.byref(Lv), ctypes.byref(Cv), valid.ctypes.data, 200, 0,
                                         -1, 0.9, 1, m_out.ctypes.data, ctypes.byref(nm)),
            "WindowSearch(window 200) (src/ORBmatcher.cc:409-516)"),
        "pair_15": (
            lambda lib_: lib_.orbx_ref_search_by_projection_pair(ctypes.byref(Lv), ctypes.byref(Cv), xyz.ctypes.data,
                                                                 valid.ctypes.data, asg.ctypes.data, T.ctypes.data,
                                                                 cam.ctypes.data, 15, ctypes.c_float(0.9),
                                                                 m_out.ctypes.data, ctypes.byref(nm)),
            lambda: L.orbx_search_by_projection_pair(ctx1.handle, ctypes.byref(Lv), ctypes.byref(Cv), xyz.ctypes.data,
                                                     valid.ctypes.data, asg.ctypes.data, T.ctypes.data,
                                                     cam.ctypes.data, 15, 0.9, m_out.ctypes.data, ctypes.byref(nm)),
            "SearchByProjection(Frame&, Frame&, window 15) (src/ORBmatcher.cc:519-594)"),
        "local_map_th1": (
            lambda lib_: lib_.orbx_ref_search_by_projection_local(ctypes.byref(Cv), len(kl), valid.ctypes.data,
                                                                  proj.ctypes.data, pred.ctypes.data, vcos.ctypes.data,
                                                                  mpd.ctypes.data, asg.ctypes.data, ctypes.c_float(1.0),
                                                                  ctypes.c_float(0.8), m_out.ctypes.data,
                                                                  ctypes.byref(nm)),
            lambda: L.orbx_search_by_projection_local(ctx1.handle, ctypes.byref(Cv), len(kl), valid.ctypes.data,
                                                      proj.ctypes.data, pred.ctypes.data, vcos.ctypes.data,
                                                      mpd.ctypes.data, asg.ctypes.data, 1.0, 0.8, m_out.ctypes.data,
                                                      ctypes.byref(nm)),
            "SearchByProjection(Frame&, local map, th 1) (src/ORBmatcher.cc:49-125)"),
    }
    ts = {}
    for name, (cpu_fn, gpu_fn, what) in searches.items():
        cpu_fn(P)
        ref = (m_out.copy(), nm.value)
        check_rc(gpu_fn(), name)
        leg = {"bit_exact": bool(np.array_equal(m_out, ref[0]) and nm.value == ref[1]), "matches": ref[1],
               "gpu": time_calls(lambda i: check_rc(gpu_fn(), name), 1, proto),
               "cpu": time_calls(lambda i: cpu_fn(R), 1, proto), "call": what}
        leg["speedup_vs_cpu"] = round(leg["cpu"]["median_ms"] / leg["gpu"]["median_ms"], 2)
        ts[name] = leg
    ts["note"] = ("host frame views of two consecutive extracted frames (1000 keypoints); candidate lists per query "
                  "across the chip, greedy assignment resolved in parallel fixed-point rounds (k_area_replay)")
    out["tracking_searches"] = ts
    ctx1.close()

    # --- one whole Tracking frame on the device (orbx_track_frame) ----------
    # TrackWithMotionModel + TrackLocalMap (src/Tracking.cc:572-627,
    # 701-752): image in, extraction, motion search, PoseOptimization,
    # frustum + local-map search, PoseOptimization, one read-back; cpu = the
    # same chain over the oracle (tests/track_data.py ref_chain)
    import track_data as td
    ctxt = ox.Context(nfeatures=nf, max_w=w, max_h=h, slots=3, device=args.device)
    last_img, cur_img = td.images(w, h, 6, 11)
    ctxt.upload(last_img, 0)
    ctxt.extract(0, 1)
    ctxt.sync()
    tkl, tdl = ctxt.features(0)
    tscene = td.make_scene(tkl, tdl, 11)
    tpred = td.pose_x(7.5 * td.DEPTH / float(td.CAM[0]))
    tq_img, tkeep_img = td.query(tscene, tpred, slot=1, image=cur_img, last_slot=0, cap=nf)
    tq_slot, tkeep_slot = td.query(tscene, tpred, slot=1, last_slot=0, cap=nf)
    check_rc(L.orbx_track_frame(ctxt.handle, ctypes.byref(tq_img)), "orbx_track_frame")
    tkc, tdc = ctxt.features(1)
    texp = td.ref_chain(P, tkl, tdl, tkc, tdc, tscene, tpred)
    tr = {}
    for exact, key in ((0, "gpu_fast_sums"), (1, "gpu")):
        check_rc(L.orbx_pose_set_exact(ctxt.handle, exact), "orbx_pose_set_exact")
        leg = {"with_extraction": time_calls(lambda i: check_rc(L.orbx_track_frame(ctxt.handle, ctypes.byref(tq_img)),
                                                                "orbx_track_frame"), 1, proto),
               "chain_only": time_calls(lambda i: check_rc(L.orbx_track_frame(ctxt.handle, ctypes.byref(tq_slot)),
                                                           "orbx_track_frame"), 1, proto)}
        got = td.result(tq_slot, tkeep_slot)
        same = all(got[k] == texp[k] for k in ("status", "n_cur", "n_motion", "n_after_pose", "n_in_view", "n_local",
                                               "n_inliers"))
        same = same and np.array_equal(got["cur_mp"], texp["cur_mp"]) and np.array_equal(got["cur_outlier"],
                                                                                         texp["cur_outlier"])
        leg["matches_identical"] = bool(same)
        leg["max_abs_tcw_diff_vs_oracle"] = float(np.abs(got["Tcw"] - texp["Tcw"]).max())
        tr[key] = leg
    # mode 1: TrackPreviousFrame then TrackLocalMap (the reference's fallback
    # after a failed motion model), on the same frames
    tq_prev, tkeep_prev = td.query(tscene, td.pose_x(0.0), slot=1, last_slot=0, cap=nf, mode=1)
    tr["previous_frame_chain_only"] = time_calls(
        lambda i: check_rc(L.orbx_track_frame(ctxt.handle, ctypes.byref(tq_prev)), "orbx_track_frame"), 1, proto)
    pgot = td.result(tq_prev, tkeep_prev)
    pexp = td.ref_chain_prev(P, tkl, tdl, tkc, tdc, tscene, td.pose_x(0.0))
    tr["previous_frame_chain_only"]["identical_to_oracle"] = bool(
        all(pgot[k] == pexp[k] for k in ("status", "n_motion", "n_pair", "n_after_pose", "n_local", "n_inliers"))
        and np.array_equal(pgot["cur_mp"], pexp["cur_mp"]) and np.array_equal(pgot["Tcw"], pexp["Tcw"]))
    ctxt.close()
    tr["cpu"] = {"with_extraction": time_calls(lambda i: (rex(cur_img), td.ref_chain(R, tkl, tdl, tkc, tdc, tscene,
                                                                                   tpred)), 1, proto),
                 "chain_only": time_calls(lambda i: td.ref_chain(R, tkl, tdl, tkc, tdc, tscene, tpred), 1, proto)}
    for k in ("with_extraction", "chain_only"):
        tr["speedup_vs_cpu_" + k] = round(tr["cpu"][k]["median_ms"] / tr["gpu"][k]["median_ms"], 2)
    tr["status"] = texp["status"]
    tr["counts"] = {k: int(texp[k]) for k in ("n_motion", "n_after_pose", "n_in_view", "n_local", "n_inliers")}
    tr["call"] = ("orbx_track_frame: one 640x480 image in (or the slot already extracted: chain_only), last frame in "
                  "its slot, local map of %d points; one upload, one read-back (cpu: the oracle's extractor, "
                  "matchers and PoseOptimization in the same order, numpy glue)" % len(tscene["pos"]))
    out["tracking_frame"] = tr

    # --- Optimizer::PoseOptimization on one frame ------------------------
    ctxp = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1, device=args.device)
    pframes = [sp.make_frame(n_kp=1000, seed=7000 * 1000 + i) for i in range(16)]
    pstructs = [sp.to_ctypes(fr) for fr in pframes]
    work = [sp.PoseFrame.from_buffer_copy(p) for p, _ in pstructs]
    ninl = ctypes.c_int()
    R.orbx_ref_pose_optimization.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]

    def pose_reset(i):
        ctypes.memmove(ctypes.addressof(work[i]), ctypes.addressof(pstructs[i][0]), ctypes.sizeof(work[i]))

    po = {"gpu": time_calls(lambda i: check_rc(L.orbx_pose_optimization(ctxp.handle, ctypes.byref(work[i]),
                                                                        ctypes.byref(ninl), None),
                                               "orbx_pose_optimization"), len(work), proto, reset=pose_reset)}
    gpu_tcw = [np.ctypeslib.as_array(work[i].Tcw).copy() for i in range(len(work))]
    po["cpu"] = time_calls(lambda i: R.orbx_ref_pose_optimization(ctypes.byref(work[i]), None, None), len(work), proto,
                           reset=pose_reset)
    P = oracle_lib.load()                     # the parity oracle for the comparison
    P.orbx_ref_pose_optimization.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    cpu_tcw = []
    for i in range(len(work)):
        pose_reset(i)
        P.orbx_ref_pose_optimization(ctypes.byref(work[i]), None, None)
        cpu_tcw.append(np.ctypeslib.as_array(work[i].Tcw).copy())
    po["max_abs_tcw_diff_vs_oracle"] = float(max(np.abs(a - b).max() for a, b in zip(gpu_tcw, cpu_tcw)))
    po["tcw_bit_identical_to_oracle"] = all(np.array_equal(a, b) for a, b in zip(gpu_tcw, cpu_tcw))
    po["speedup_vs_cpu"] = round(po["cpu"]["median_ms"] / po["gpu"]["median_ms"], 2)
    # the opt-in fast sums (orbx_pose_set_exact(ctx, 0)): lane-strided
    # partials through a fixed tree, poses within 1e-5
    check_rc(L.orbx_pose_set_exact(ctxp.handle, 0), "orbx_pose_set_exact")
    po["gpu_fast_sums"] = time_calls(lambda i: check_rc(L.orbx_pose_optimization(ctxp.handle, ctypes.byref(work[i]),
                                                                                 ctypes.byref(ninl), None),
                                                        "orbx_pose_optimization"), len(work), proto, reset=pose_reset)
    fast_tcw = [np.ctypeslib.as_array(work[i].Tcw).copy() for i in range(len(work))]
    check_rc(L.orbx_pose_set_exact(ctxp.handle, 1), "orbx_pose_set_exact")
    po["gpu_fast_sums"]["max_abs_tcw_diff_vs_oracle"] = float(max(np.abs(a - b).max()
                                                                  for a, b in zip(fast_tcw, cpu_tcw)))
    po["call"] = ("orbx_pose_optimization: one frame, 1000 keypoints, ~700 map-point edges, ~10 % outliers "
                  "(Optimizer::PoseOptimization, src/Optimizer.cc:154-285)")
    out["pose_optimization"] = po
    ctxp.close()

    # --- Optimizer::LocalBundleAdjustment on one problem -------------------
    ctxb = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1, device=args.device)
    probs = [sb.make_problem(n_kf=20, n_points=2000, seed=5000 * 1000 + i) for i in range(4)]
    bwork = [sb.to_ctypes(pr) for pr in probs]
    es = [np.zeros(p.n_edges, np.uint8) for p, _ in bwork]
    pb = [np.zeros(p.n_points, np.uint8) for p, _ in bwork]
    R.orbx_ref_lba.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p]

    def lba_reset(i):
        a, pr = bwork[i][1], probs[i]
        np.copyto(a["pose_q"], pr["pose_q"])
        np.copyto(a["pose_t"], pr["pose_t"])
        np.copyto(a["points"], pr["points"])

    st = sb.BAStats()
    ba = {"gpu": time_calls(lambda i: check_rc(L.orbx_lba_solve(ctxb.handle, ctypes.byref(bwork[i][0]), 5, 10, None,
                                                                es[i].ctypes.data, pb[i].ctypes.data,
                                                                ctypes.byref(st)), "orbx_lba_solve"),
                            len(bwork), proto, reset=lba_reset)}
    gq = [bwork[i][1]["pose_q"].copy() for i in range(len(bwork))]
    ba["cpu"] = time_calls(lambda i: R.orbx_ref_lba(ctypes.byref(bwork[i][0]), 5, 10, es[i].ctypes.data,
                                                    pb[i].ctypes.data, ctypes.byref(st)),
                           len(bwork), proto, reset=lba_reset)
    P.orbx_ref_lba.argtypes = R.orbx_ref_lba.argtypes
    worst = 0.0
    for i in range(len(bwork)):
        lba_reset(i)
        P.orbx_ref_lba(ctypes.byref(bwork[i][0]), 5, 10, es[i].ctypes.data, pb[i].ctypes.data, ctypes.byref(st))
        worst = max(worst, float(np.abs(gq[i] - bwork[i][1]["pose_q"]).max()))
    ba["max_abs_pose_q_diff_vs_oracle"] = worst
    ba["speedup_vs_cpu"] = round(ba["cpu"]["median_ms"] / ba["gpu"]["median_ms"], 2)
    ba["call"] = ("orbx_lba_solve: one 20 KF (+2 fixed) x 2000 MP problem, optimize(5), outlier pass, optimize(10), "
                  "outlier pass (Optimizer::LocalBundleAdjustment, src/Optimizer.cc:287-536)")
    out["lba_solve"] = ba
    ctxb.close()

    # --- ORB-SLAM's three threads at once on this GPU ----------------------
    # Tracking (extract -> motion search -> pose), LocalMapping (local BA over
    # several workgroups -> triangulation search) and LoopClosing (BoW search
    # -> Sim3 search), each on its own context and host thread
    # (src/main.cc:122-133; tests/test_threads_gpu.py): per-call medians one
    # thread at a time and under contention, outputs compared bit for bit
    import threads_work as tw
    tin = tw.make_inputs()
    tcs = tw.make_contexts()
    rounds = 40
    alone_o = {k: [] for k in tw.WORK}
    alone_t = {k: [] for k in tw.WORK}
    for k in tw.WORK:
        for r in range(rounds):
            o, t = tw.WORK[k](tcs[k], tin, r)
            alone_o[k].append(o)
            alone_t[k].append(t)
    res, conc_t, errs = tw.run_threads(tcs, tin, rounds)
    same = not errs and all(tw.same(o, alone_o[k][r]) for k in tw.WORK for r, o in enumerate(res[k]))
    lba_wg = L.orbx_lba_last_workgroups(tcs["local_mapping"].handle)
    for c in tcs.values():
        c.close()
    out["three_threads"] = {
        "median_ms_alone": tw._medians(alone_t), "median_ms_concurrent": tw._medians(conc_t),
        "rounds_per_thread": rounds, "outputs_identical_to_alone": bool(same), "errors": errs,
        "lba_workgroups": lba_wg,
        "note": "Tracking / LocalMapping / LoopClosing calls from three host threads, one context each "
                "(src/main.cc:122-133); local BA on the multi-workgroup kernel (plain launch, residency cap)"}
    return out


def host_inclusive_frames(args, ctx, frames, B, bf, configure):
    """c2 with the host boundary inside the timed region: each step uploads
    its B frames from page-locked host memory (orbx_dev_upload_async, the next
    step's frames while this step extracts), extracts + matches them, and
    reads keypoints, descriptors, counts and match vectors back into
    page-locked host memory (orbx_dev_download_async).  Reported beside
    `value`, never as it (the task's contract keeps inputs resident there)."""
    h, w = frames.shape[1:]
    nf = ctx.nfeatures
    src = ox.HostArray((B, h, w), np.uint8)
    src.array[:] = frames
    outs = [dict(kps=ox.HostArray((B * nf,), ox.KEYPOINT), desc=ox.HostArray((B * nf, 32), np.uint8),
                 n=ox.HostArray((B,), np.int32), m12=ox.HostArray((B * nf,), np.int32),
                 nm=ox.HostArray((B,), np.int32)) for _ in range(2)]
    configure(False)
    it = [0]

    def step():
        k = it[0]
        it[0] += 1
        first, nxt = (k % 2) * B, ((k + 1) % 2) * B
        ctx.upload_async(src.array, first=nxt)       # next step's frames, behind this step's extraction
        ctx.extract_match(first, B, B, mode="bf" if bf else "init", window=100, th_low=50, nnratio=0.9,
                          check_ori=True)
        o = outs[k % 2]
        ctx.download_async(first, B, o["kps"].array, o["desc"].array, o["n"].array, o["m12"].array, o["nm"].array)

    ctx.upload_async(src.array, first=0)
    for _ in range(args.warmup):
        step()
    ctx.sync()
    steps = max(5, args.steps)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.sync()
    dt = time.perf_counter() - t0
    # the last step's host buffers against the device-resident outputs (which
    # parity_frames checks against the oracle)
    k = it[0] - 1
    first, o = (k % 2) * B, outs[k % 2]
    bad = []
    for f in (0, B // 2, B - 1):
        gk, gd = ctx.features(first + f)
        gm, gn = ctx.matches(first + f)
        hk = o["kps"].array[f * nf:f * nf + len(gk)]
        ok = (int(o["n"].array[f]) == len(gk) and np.array_equal(hk.view(np.uint8), gk.view(np.uint8))
              and np.array_equal(o["desc"].array[f * nf:f * nf + len(gk)], gd)
              and int(o["nm"].array[f]) == gn and np.array_equal(o["m12"].array[f * nf:(f + 1) * nf], gm))
        if not ok:
            bad.append(first + f)
    in_b = B * h * w
    out_b = B * (nf * (28 + 32 + 4) + 8)
    res = {"frames_per_s": round(B * steps / dt, 2), "ms_per_step": round(1e3 * dt / steps, 4), "steps": steps,
           "h2d_GBps": round(in_b * steps / dt / 1e9, 2), "d2h_GBps": round(out_b * steps / dt / 1e9, 2),
           "host_buffers_equal_device_outputs": not bad,
           "boundary": "images uploaded from page-locked host memory and keypoints / descriptors / counts / match "
                       "vectors read back into it inside the timed region (orbx_dev_upload_async, "
                       "orbx_dev_download_async)"}
    for o in outs:
        for v in o.values():
            v.close()
    src.close()
    return res


def parity_frames(ctx, frames, first, B, nf, w, h, bf):
    """Bit-exact check of the last timed step's output against the oracle
    (run after the timed region, with the CPU baseline): the pipeline's part
    boundaries and a few interior frames of slot range [first, first + B),
    keypoints + descriptors and the match vector against the predecessor."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    L = oracle_lib.load()
    era = ctx.nth_pivot()        # retainBest's libstdc++ era the product ran (orbx_get_nth_pivot)
    ex = oracle_lib.RefExtractor(nf, nth_pivot=era)
    ways = 3
    picks = sorted({min(B - 1, max(0, v)) for i in range(ways) for v in (B * i // ways, B * (i + 1) // ways - 1)}
                   | {B // 2})
    ref = {}
    bad = []
    for f in picks:
        for g in ((f - 1) % B, f):
            if g not in ref:
                ref[g] = ex(frames[g])
        rk, rd = ref[f]
        pk, pd = ref[(f - 1) % B]
        gk, gd = ctx.features(first + f)
        gm, gn = ctx.matches(first + f)
        ok = np.array_equal(gk.view(np.uint8), rk.view(np.uint8)) and np.array_equal(gd, rd)
        if bf:
            bi, b1, b2 = (np.zeros(len(pd), np.int32) for _ in range(3))
            L.orbx_ref_hamming_bf(oracle_lib.ptr(pd), len(pd), oracle_lib.ptr(rd), len(rd), oracle_lib.ptr(bi),
                                  oracle_lib.ptr(b1), oracle_lib.ptr(b2))
            want = np.where((b1 <= 50) & (b1.astype(np.float32) < b2.astype(np.float32) * np.float32(0.9)), bi, -1)
            wn = int((want >= 0).sum())
        else:
            F1, F2 = ox.frame_view(pk, pd, w, h), ox.frame_view(rk, rd, w, h)
            pm = np.stack([pk["x"], pk["y"]], 1).astype(np.float32).copy()
            want = np.zeros(len(pk), np.int32)
            nm = ctypes.c_int()
            L.orbx_ref_search_for_initialization(ctypes.byref(F1), ctypes.byref(F2), oracle_lib.ptr(pm),
                                                 oracle_lib.ptr(want), 100, 0.9, 1, ctypes.byref(nm))
            wn = nm.value
        ok = ok and gn == wn and np.array_equal(gm[:len(pk)], want)
        if not ok:
            bad.append(first + f)
    return {"bit_exact": not bad, "slots": [first + f for f in picks], "mismatched_slots": bad,
            "oracle": "oracle/liborbx_ref.so", "what": "keypoints, descriptors and matches of the last timed step",
            "nth_element_era": {1: "GCC 4.6-4.8 (ORBX_NTH_PIVOT_GCC48, the default)",
                                0: "GCC >= 4.9 (ORBX_NTH_PIVOT_GCC49)"}[era]}


def run_frames(args, wl, rank, local, world, dist):
    w, h, nf, B = wl["w"], wl["h"], wl["nfeatures"], args.batch or wl["batch"]
    bf = args.workload == "c3"
    frames = synth.sequence(w, h, B, seed=odist.shard_seed(2000, rank))
    # two slot ranges: step k extracts range k % 2 while the matching of
    # step k - 1 (the other range) finishes on the context's match stream
    ctx = ox.Context(nfeatures=nf, max_w=w, max_h=h, slots=2 * B, device=args.device)
    ctx.upload(frames, first=0)
    ctx.upload(frames, first=B)
    if args.split_ways:
        ctx.set_split(args.split_ways)
    pipelined = not (args.sync_match or args.serial)

    def configure(serial):
        ctx.set_split(0 if serial else (args.split_ways or 1))
        ctx.set_async_match(not serial and pipelined)

    configure(args.serial)
    it = [0]
    last = [0]

    def step():
        first = (it[0] % 2) * B
        last[0] = first
        it[0] += 1
        if args.sync_match:   # extraction, then matching, in order on the context stream
            ctx.extract(first, B)
            if bf:
                ctx.match_bf_prev(first, B, B, th_low=50, nnratio=0.9)
            else:
                ctx.match_prev(first, B, B, window=100, nnratio=0.9, check_ori=True)
            return
        ctx.extract_match(first, B, B, mode="bf" if bf else "init", window=100, th_low=50, nnratio=0.9,
                          check_ori=True)

    for _ in range(args.warmup):
        step()
    ctx.sync()
    names = ["pyr0", "resize", "fast", "retain", "blur", "describe", "match"]
    if args.serial:
        # diagnostic form (PMC collection of the serialised launches): the
        # timed steps themselves run one launch per kernel over the batch
        elapsed, kernels = timed(args, ctx, step, dist, names)
        kernels = {"timed": None, "serial": kernels, "serial_steps": args.steps}
    else:
        # Serialised pass before the timed region (3 steps: one launch per
        # kernel over the whole batch, matching in order, every kernel timed):
        # the per-kernel breakdown and the headline roofline; then the
        # pipelined timed steps carry events on the dominant kernel only.
        iso = {}
        dominant = "fast"
        if not args.no_isolated:
            configure(True)
            iso_args = argparse.Namespace(**{**vars(args), "steps": 3, "no_kernel_timing": False})
            _, iso = timed(iso_args, ctx, step, None, names)
            configure(False)
            dominant = max(iso, key=lambda k: iso[k]["total_ms"])
            for _ in range(args.warmup):
                step()
            ctx.sync()
        elapsed, kernels = timed(args, ctx, step, dist, [dominant], only=dominant)
        kernels = {"timed": kernels, "serial": iso or None, "serial_steps": 3}
    k0, _ = ctx.features(B - 1)
    _, nm = ctx.matches(B - 1)
    stats = np.array([elapsed, B * args.steps, len(k0), nm], dtype=np.float64)
    allst = odist.gather_stats(stats, dist, device=args.gather_device)   # before rank 0's CPU legs
    ab = algorithmic_bytes(w, h, nf, "bf" if bf else "init")
    units_per_step = {k: B for k in ab}
    cpu = None
    check = {"last_frame_keypoints": int(stats[2]), "last_frame_matches": int(stats[3])}
    if rank == 0 and not args.no_cpu_baseline:
        check["parity_last_step"] = parity_frames(ctx, frames, last[0], B, nf, w, h, bf)
        L, desc = native_oracle()
        cpu = cpu_baseline_frames(frames, nf, CPU_PROTOCOL[args.workload], bf=bf, L=L, lib_desc=desc)
        cpu["all_cores"] = cpu_all_cores_frames(frames, nf, max(3.0, args.cpu_budget / 2), bf=bf, L=L, lib_desc=desc)
    if rank == 0 and not args.no_host_inclusive and not args.serial:
        check["host_inclusive"] = host_inclusive_frames(args, ctx, frames, B, bf, configure)
    if rank == 0 and world == 1 and args.workload == "c2" and not (args.no_single_call or args.no_cpu_baseline):
        check["single_call"] = single_call_legs(args, frames, nf, w, h)
    cfg = {"workload": wl["desc"], "frames_per_step_per_gpu": B, "nfeatures": nf, "image": f"{w}x{h}",
           "parallelism": f"dp{world} (one sequence per GPU)",
           "pipeline": ("serialised (diagnostic --serial)" if args.serial else
                        "sync matching" if args.sync_match else
                        f"{args.split_ways or 3}-part extraction pipeline, asynchronous matching")}
    ctx.close()
    return allst, kernels, ab, units_per_step, cpu, check, cfg


def parity_lba(uniq, work, es, pb, st, sample=(0, 1, 2, 3)):
    """The last timed run's fetched results of a few problems against the
    oracle LBA: poses within 1e-5 (north_star), points 1e-4, identical
    outlier decisions and LM iteration counts."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    from orb_slam_amd import synth_ba as sb
    L = oracle_lib.load()
    L.orbx_ref_lba.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p]
    worst, bad = 0.0, []
    for i in sample:
        p, arrs = sb.to_ctypes(uniq[i])
        res = np.zeros(p.n_edges, np.uint8)
        rpb = np.zeros(p.n_points, np.uint8)
        rst = sb.BAStats()
        L.orbx_ref_lba(ctypes.byref(p), 5, 10, res.ctypes.data, rpb.ctypes.data, ctypes.byref(rst))
        g = work[i][1]
        d = max(float(np.abs(g["pose_q"] - arrs["pose_q"]).max()), float(np.abs(g["pose_t"] - arrs["pose_t"]).max()))
        worst = max(worst, d)
        same = (np.array_equal(es[i], res) and np.array_equal(pb[i], rpb)
                and list(st[i].iterations) == list(rst.iterations)
                and float(np.abs(g["points"] - arrs["points"]).max()) <= 1e-4)
        if d > 1e-5 or not same:
            bad.append(i)
    return {"within_1e-5": not bad, "max_abs_pose_diff": worst, "problems": list(sample), "mismatched": bad,
            "oracle": "oracle/liborbx_ref.so"}


def run_lba(args, wl, rank, local, world, dist):
    from orb_slam_amd import synth_ba as sb
    P = args.batch or wl["batch"]
    # 32 distinct synthetic problems (generation is slow in Python), repeated
    # to fill the batch; every problem is solved independently from its own copy
    uniq = [sb.make_problem(n_kf=20, n_points=2000, seed=odist.shard_seed(5000, rank) * 1000 + i)
            for i in range(min(P, 32))]
    probs = [uniq[i % len(uniq)] for i in range(P)]
    ctx = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1, device=args.device)
    L = ox.lib()
    # host-side problem arrays, marshalled once
    work = [sb.to_ctypes(pr) for pr in probs]
    n_edges = int(np.mean([c[0].n_edges for c in work]))
    arr = (sb.BAProblem * P)(*[c[0] for c in work])
    es = [np.zeros(c[0].n_edges, np.uint8) for c in work]
    pb = [np.zeros(c[0].n_points, np.uint8) for c in work]
    esp = (ctypes.c_void_p * P)(*[e.ctypes.data for e in es])
    pbp = (ctypes.c_void_p * P)(*[b.ctypes.data for b in pb])

    def check_rc(r, where):
        if r != 0:
            raise ox.OrbxError(r, where)

    # the problems are staged in HBM before the timed region; every run
    # restarts from the staged state (orbx_lba_stage / orbx_lba_run)
    check_rc(L.orbx_lba_stage(ctx.handle, P, arr), "orbx_lba_stage")

    def step():
        check_rc(L.orbx_lba_run(ctx.handle, 5, 10, None), "orbx_lba_run")

    for _ in range(args.warmup):
        step()
    elapsed, kernels = timed(args, ctx, step, dist, ["lba_iter", "lba_outliers"])
    kernels = {"timed": None, "serial": kernels, "serial_steps": args.steps}   # one stream, in order
    st = (sb.BAStats * P)()
    check_rc(L.orbx_lba_fetch(ctx.handle, arr, esp, pbp, st), "orbx_lba_fetch")
    cpu_leg = rank == 0 and not args.no_cpu_baseline
    stats = np.array([elapsed, P * args.steps, st[0].iterations[0] + st[0].iterations[1], st[0].n_outliers[0]],
                     dtype=np.float64)
    allst = odist.gather_stats(stats, dist, device=args.gather_device)   # before rank 0's CPU legs
    # the last timed run's results against the oracle, before the host-array
    # leg below reuses these arrays (after the gather: the other ranks do
    # not wait in the collective while rank 0 runs the oracle)
    parity = parity_lba(uniq, work, es, pb, st) if cpu_leg else None
    # the host-array boundary (orbx_lba_solve_batch: packing, H2D upload,
    # both passes, D2H readback and unpacking), timed beside it on rank 0;
    # reported in `check`, never as `value`
    pcie = None
    if rank == 0:
        def host_step():
            for (_, a), pr in zip(work, probs):
                np.copyto(a["pose_q"], pr["pose_q"])
                np.copyto(a["pose_t"], pr["pose_t"])
                np.copyto(a["points"], pr["points"])
            check_rc(L.orbx_lba_solve_batch(ctx.handle, P, arr, 5, 10, None, esp, pbp, (sb.BAStats * P)()),
                     "orbx_lba_solve_batch")
        host_step()
        n_host = max(3, args.steps // 4)
        t0 = time.perf_counter()
        for _ in range(n_host):
            host_step()
        dt = time.perf_counter() - t0
        pcie = {"problems_per_s": round(P * n_host / dt, 2), "ms_per_step": round(1e3 * dt / n_host, 3),
                "steps": n_host, "boundary": "orbx_lba_solve_batch: host arrays in / out (packing, H2D, D2H)"}
    ab = {"lba_iter": lba_bytes(22, 2000, n_edges), "lba_outliers": n_edges * 16}
    # lba_bytes is per problem and LM iteration: the two lba_iter launches of
    # a step run the 5 and the 10 iterations of all P problems (one launch per
    # optimize() pass without abort flags), lba_outliers one pass over all P
    # (2 per step)
    units_per_step = {"lba_iter": P * 15, "lba_outliers": P * 2}
    cpu = None
    flops = float(sum(lba_flops(probs[i], st[i]) for i in range(P)))
    check = {"iterations_problem0": int(stats[2]), "outliers_pass1_problem0": int(stats[3]),
             "edges_per_problem": n_edges, "pcie_inclusive": pcie, "fp64_flops_per_step": flops}
    if cpu_leg:
        check["parity_last_step"] = parity
        L, desc = native_oracle()
        cpu = cpu_baseline_lba(probs, CPU_PROTOCOL["c5"], L=L, lib_desc=desc)
        cpu["all_cores"] = cpu_all_cores_lba(probs, max(3.0, args.cpu_budget / 2), L=L, lib_desc=desc)
    cfg = {"workload": wl["desc"], "problems_per_step_per_gpu": P, "keyframes": 20, "map_points": 2000,
           "parallelism": f"dp{world} (independent problems per GPU; replicas)",
           "boundary": "problems staged in HBM before the timed region (orbx_lba_stage); results fetched after"}
    ctx.close()
    return allst, kernels, ab, units_per_step, cpu, check, cfg


# bench timer name -> kernel symbol in the rocprofv3 CSVs
KERNEL_SYMBOL = {"pyr0": "k_pyr_level0", "resize": ("k_pyr_resize", "k_pyr_cascade"), "fast": "k_fast_cells",
                 "retain": "k_retain_cells", "blur": "k_blur", "describe": "k_describe",
                 "match": "k_match_", "lba_iter": "k_lba_iteration", "lba_outliers": "k_lba_outliers",
                 "pose": "k_pose_opt"}


def pmc_summary(key):
    """Newest committed PMC summary of bench command `key`
    (profiles/rNN_<key>_pmc_hbm.json, tools/pmc_summary.py: separate
    FETCH_SIZE / WRITE_SIZE / SQ passes).  key = <workload> for the pipelined
    bench command, <workload>_serial for `bench.py --serial` (one launch per
    kernel over the whole batch).  Returns (summary, source) only when the
    profile names the liborbx.so loaded now (SHA-256), else (None, note)."""
    import hashlib
    cands = sorted((ROOT / "profiles").glob(f"r*_{key}_pmc_hbm.json"))
    if not cands:
        return None, None
    summary = json.loads(cands[-1].read_text())
    meta = summary.pop("_meta", {})
    if meta.get("liborbx_sha256") != hashlib.sha256(Path(ox.LIB_PATH).read_bytes()).hexdigest():
        return None, f"profiles/{cands[-1].name}: profile of another liborbx.so build (SHA-256 differs), not reported"
    return summary, f"profiles/{cands[-1].name} (per dispatch, build {meta.get('git_head')})"


def pmc_traffic(key, name):
    """HBM bytes per launch of kernel `name`: FETCH_SIZE x2 (gfx950 wide-read
    correction, MI355X_MICROARCH.md HBM section) + WRITE_SIZE as `traffic`,
    FETCH_SIZE + WRITE_SIZE as counted as `traffic_raw`."""
    summary, src = pmc_summary(key)
    sym = KERNEL_SYMBOL.get(name)
    if summary is None or not sym:
        return {"traffic": None, "traffic_source": src}
    syms = sym if isinstance(sym, tuple) else (sym,)
    hits = [v for k, v in summary.items() if any(s in k for s in syms)]
    if not hits:
        return {"traffic": None, "traffic_source": src}
    return {"traffic": round(sum(h["hbm_bytes_fetch_x2"] for h in hits) / len(hits)),
            "traffic_raw": round(sum(h["hbm_bytes_raw"] for h in hits) / len(hits)),
            "traffic_source": src + ", FETCH_SIZE x2 + WRITE_SIZE (traffic_raw: FETCH_SIZE + WRITE_SIZE)"}


# wave64 VALU issue peak: 256 CUs x 4 SIMDs, one wave64 instruction per 2
# cycles per SIMD (32 lanes), 2.4 GHz (MI355X_MICROARCH.md constants table)
VALU_PEAK_TIPS = 256 * 4 * 2.4e9 / 2 / 1e12


def pmc_valu(key, name):
    """SQ_INSTS_VALU per launch of kernel `name` from the same summary."""
    summary, src = pmc_summary(key)
    sym = KERNEL_SYMBOL.get(name)
    if summary is None or not sym:
        return None
    syms = sym if isinstance(sym, tuple) else (sym,)
    hits = [v["SQ_INSTS_VALU"] for k, v in summary.items() if any(s in k for s in syms) and "SQ_INSTS_VALU" in v]
    if not hits:
        return None
    return {"insts_per_launch": sum(hits) / len(hits), "source": src + " SQ_INSTS_VALU"}


def timed(args, ctx, step, dist, names, only=None):
    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            if torch.cuda.device_count():   # the stubbed-context CPU test has no GPU
                torch.cuda.synchronize()

    ctx.timing(not args.no_kernel_timing, only=only)
    barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    kernels = {}
    for name in names:
        n, avg, tot = ctx.kernel_time(name)
        kernels[name] = {"launches": n, "avg_ms": avg, "total_ms": tot}
    ctx.timing(False)
    return elapsed, kernels


def spawn_ranks(n):
    """`bench.py --gpus N` without a torchrun environment: start N rank
    processes of this same script (sys.argv[0], so a wrapper that installs a
    test context is re-entered too) with RANK / LOCAL_RANK / WORLD_SIZE and a
    127.0.0.1 rendezvous, before this process makes any GPU call, and return
    the first non-zero exit code (the others are then terminated by pid)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(sys.argv[0]), *sys.argv[1:]], env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:
                    q.terminate()
        time.sleep(0.05)
    return rc


def init_ranks(world, local):
    """Process group for N > 1 ranks: RCCL ("nccl") when every rank has a GPU
    of its own, gloo otherwise (N ranks sharing one GPU, as on a 1-GPU box,
    or no GPU at all: the CPU tests).  torch.cuda.device_count() does not
    initialise the GPU on this image.  Returns (dist, device index for the
    orbx context, device of the stats gather)."""
    import torch
    import torch.distributed as tdist
    ngpu = odist.visible_gpus()
    backend = os.environ.get("ORBX_BENCH_BACKEND") or ("nccl" if ngpu >= world else "gloo")
    device = local % ngpu if ngpu else 0
    if ngpu:
        torch.cuda.set_device(device)
    # gloo announces its connections on stdout from C++; stdout carries the
    # one JSON line, so the process group is set up with fd 1 on stderr
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        tdist.init_process_group(backend)
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    return tdist, device, ("cuda" if backend == "nccl" else "cpu")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0, help="frames (or BA problems) per step per GPU")
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-budget", type=float, default=12.0,
                    help="seconds of the all-cores CPU baseline x2 (the 1-core baseline follows CPU_PROTOCOL)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-protocol", default="",
                    help="W,T: CPU baseline warm-up and timed units (default CPU_PROTOCOL: SURVEY.md 8(d)'s 50,500)")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--no-isolated", action="store_true",
                    help="skip the serialised per-kernel pass after the timed steps (PMC collection)")
    ap.add_argument("--sync-match", action="store_true",
                    help="match each batch after its extraction on the same stream (no overlap with the next "
                         "batch's extraction)")
    ap.add_argument("--serial", action="store_true",
                    help="diagnostic: time serialised steps (one launch per kernel over the batch, matching in "
                         "order) -- the form the headline roofline's PMC profile is collected from")
    ap.add_argument("--split-ways", type=int, default=0, choices=[0, 2, 3, 4],
                    help="extraction pipeline parts (orbx_dev_set_split; 0 = library default, 3)")
    ap.add_argument("--pose-fast-sums", action="store_true",
                    help="pose workload: the opt-in lane-strided sums (orbx_pose_set_exact(ctx, 0))")
    ap.add_argument("--no-single-call", action="store_true",
                    help="skip the single-call latency legs of the c2 line (check.single_call)")
    ap.add_argument("--no-host-inclusive", action="store_true",
                    help="skip the host-fed throughput leg of c2 / c3 (check.host_inclusive)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="diagnostic: no per-kernel hipEvents in the timed region (roofline then unavailable)")
    args = ap.parse_args()
    if args.cpu_protocol:
        CPU_PROTOCOL[args.workload] = tuple(int(v) for v in args.cpu_protocol.split(","))

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world, rank, local = odist.env()
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    dist = None
    args.device, args.gather_device = 0, "cpu"
    if world > 1:
        dist, args.device, args.gather_device = init_ranks(world, local)
    args.dist_backend = dist.get_backend() if dist is not None else None

    wl = WORKLOADS[args.workload]
    run = {"c5": run_lba, "pose": run_pose}.get(args.workload, run_frames)
    allst, kernels, ab, units, cpu, check, cfg = run(args, wl, rank, local, world, dist)
    value, elapsed, _ = odist.job_rate(allst)

    if rank == 0:
        frames_wl = args.workload in ("c2", "c3")

        def roofline_events(kern, steps):
            # dominant kernel: largest total time; its algorithmic bytes per
            # launch (bytes per unit x units per step / launches per step) over
            # its mean launch duration (HIP events on the stream it is launched on)
            timed_k = [k for k in kern if kern[k]["launches"]] or list(kern)
            dom = max(timed_k, key=lambda k: kern[k]["total_ms"])
            launches_per_step = max(1, kern[dom]["launches"] // steps)
            per_launch = ab.get(dom, 0) * units.get(dom, 1) / launches_per_step
            avg_s = kern[dom]["avg_ms"] / 1e3
            achieved = per_launch / avg_s / 1e9 if avg_s > 0 and per_launch > 0 else 0.0
            return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None, "kernel": dom,
                    "algorithmic_bytes_per_launch": per_launch, "avg_launch_ms": kern[dom]["avg_ms"]}

        def valu_roof(key, roof):
            valu = pmc_valu(key, roof["kernel"])
            if not valu or not roof.get("avg_launch_ms"):
                return None
            rate = valu["insts_per_launch"] / (roof["avg_launch_ms"] / 1e3)
            return {"bound": "valu-issue", "achieved": round(rate / 1e12, 4), "peak": VALU_PEAK_TIPS,
                    "unit": "T wave-instr/s", "frac": round(rate / 1e12 / VALU_PEAK_TIPS, 4), "kernel": roof["kernel"],
                    "valu_insts_per_launch": valu["insts_per_launch"],
                    "valu_insts_per_frame": (valu["insts_per_launch"] / roof["frames_per_launch"]
                                             if roof.get("frames_per_launch") else None),
                    "avg_launch_ms": roof["avg_launch_ms"], "source": valu["source"]}

        roof, occ, roof_valu = None, None, None
        if kernels["serial"]:
            # the headline roofline: the dominant kernel launched alone over the
            # whole batch (the serialised pass; PMC of `bench.py --serial`)
            serial_key = f"{args.workload}_serial" if frames_wl else args.workload
            roof = roofline_events(kernels["serial"], kernels["serial_steps"])
            roof.update(pmc_traffic(serial_key, roof["kernel"]))
            if frames_wl:
                roof["frames_per_launch"] = units[roof["kernel"]] // max(
                    1, kernels["serial"][roof["kernel"]]["launches"] // kernels["serial_steps"])
                roof["launch"] = "serialised: one launch per kernel over the batch (no other kernel running)"
            roof_valu = valu_roof(serial_key, roof)
        if kernels["timed"]:
            # the same kernel inside the pipelined timed steps: its hipEvent
            # duration includes CU time shared with the other streams' kernels,
            # so this measures co-scheduling as much as the kernel
            occ = roofline_events(kernels["timed"], args.steps)
            occ.update(pmc_traffic(args.workload, occ["kernel"]))
            occ["launch"] = "overlapped: one pipeline part, concurrent with the other parts' kernels and matching"
            occ["launches_per_step"] = kernels["timed"][occ["kernel"]]["launches"] // args.steps
            if roof is None:
                roof = occ
        path = None
        if frames_wl:
            # the whole path: algorithmic bytes of every stage per step over the
            # measured step time
            step_s = elapsed / args.steps
            per_frame = survey_frame_bytes(wl["w"], wl["h"], wl["nfeatures"])
            per_step = per_frame * units["fast"] * world          # every rank's frames
            stage_step = sum(ab[k] * units[k] for k in ab) * world
            gbs = per_step / step_s / 1e9
            path = {"bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(gbs / HBM_PEAK_GBS, 5), "algorithmic_bytes_per_frame": per_frame,
                    "algorithmic_bytes_per_step": per_step,
                    "note": "SURVEY.md 8(d) B_frame (pyramid read + write, FAST read, blur read + write, outputs) x "
                            "frames per step of all ranks / ms_per_step",
                    "with_every_stage_bytes": {"bytes_per_step": stage_step,
                                               "achieved": round(stage_step / step_s / 1e9, 2),
                                               "note": "also the level-0 copy and describe's patch reads "
                                                       "(the per-kernel figures of algorithmic_bytes())"}}
        out = {
            "metric": wl["metric"], "value": round(value, 2), "unit": wl["unit"], "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64" if args.workload in ("c5", "pose") else "u8",
            "data": "synthetic (orb_slam_amd/synth.py / synth_ba.py / synth_pose.py, seeded per rank)",
            "config": cfg, "roofline": roof, "cpu_baseline": cpu, "check": check,
            "hip_hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"]),
        }
        if world > 1:
            # what `value` is made of: every rank's units and timed seconds
            # (value = sum of units / max of seconds), and how the ranks met
            out["ranks"] = {"backend": args.dist_backend, "gpus_visible": odist.visible_gpus(),
                            "elapsed_s": [round(float(x), 6) for x in allst[:, 0]],
                            "units": [int(x) for x in allst[:, 1]]}
        if occ is not None and occ is not roof:
            out["occupancy"] = occ
        if path:
            out["path_roofline"] = path
        if roof_valu:
            out["roofline_valu"] = roof_valu
        if cpu and "all_cores" in cpu:
            # the same oracle on every host core of the box
            # (one independent stream per thread), core count stated
            out["cpu_baseline_all_cores"] = cpu.pop("all_cores")
        if args.workload == "c5" and kernels["serial"] and kernels["serial"].get("lba_iter", {}).get("total_ms"):
            # FP64 vector roofline of the LM iterations (SURVEY.md 8(d) flop
            # formula over the step's iterations and trials) beside the HBM one
            it_s = kernels["serial"]["lba_iter"]["total_ms"] / 1e3 / kernels["serial_steps"]
            fl = check["fp64_flops_per_step"] / it_s / 1e12
            out["roofline_fp64"] = {"bound": "fp64-valu", "achieved": round(fl, 4), "peak": FP64_PEAK_TFLOPS,
                                    "unit": "TFLOP/s", "frac": round(fl / FP64_PEAK_TFLOPS, 5), "kernel": "lba_iter",
                                    "flops_per_step": check["fp64_flops_per_step"],
                                    "lba_iter_ms_per_step": round(it_s * 1e3, 4),
                                    "note": "algorithmic flops (SURVEY.md 8(d)): the kernel also rebuilds each edge's "
                                            "Hpl block where it is used instead of storing it"}
        if args.workload == "pose" and roof and roof.get("avg_launch_ms"):
            # PoseOptimization is FP64-VALU bound (its edges are read from HBM
            # once and kept in LDS): the FP64 roofline is the headline one, the
            # HBM figure is kept beside it
            fl = check["fp64_flops_per_frame"] * units["pose"] / (roof["avg_launch_ms"] / 1e3) / 1e12
            out["roofline_hbm"] = roof
            out["roofline"] = {"bound": "fp64-valu", "achieved": round(fl, 3), "peak": FP64_PEAK_TFLOPS,
                               "unit": "TFLOP/s", "frac": round(fl / FP64_PEAK_TFLOPS, 5),
                               "traffic": roof.get("traffic"), "kernel": roof["kernel"],
                               "flops_per_frame": check["fp64_flops_per_frame"],
                               "avg_launch_ms": roof["avg_launch_ms"]}
        if args.verbose:
            out["kernels"] = kernels
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
