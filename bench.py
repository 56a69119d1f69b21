"""Benchmark: frames/sec ORB extract+match (640x480, 1000 kp) on MI355X.

Workload (BASELINE.json configs[1]): synthetic 640x480
mono8 "TUM-style" sequences (one per rank, already resident in HBM), 8-level
pyramid, 1000 keypoints.  One step = one batch of B frames: ORB extraction of
every frame (ORBextractor::operator()) plus SearchForInitialization of every
frame against its predecessor (window 100, nnratio 0.9, orientation check;
the sequence is treated as cyclic so every frame is matched).

Multi-GPU: one process per GPU (torchrun); each rank owns its sequence; the
only collective is the end-of-run gather of stats (RCCL).  Weak scaling.

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

import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import dist as odist, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)

WORKLOADS = {
    "c2": dict(w=640, h=480, nfeatures=1000, desc="640x480 mono8, 8 levels x1.2, 1000 kp: ORB extract + "
               "SearchForInitialization vs previous frame"),
    "c3": dict(w=1920, h=1080, nfeatures=2000, desc="1920x1080 mono8, 8 levels x1.2, 2000 kp: ORB extract + "
               "SearchForInitialization vs previous frame"),
}


def level_sizes(w, h, nlevels=8, scale=1.2):
    sizes = []
    invf = np.float32(1.0 / np.float64(np.float32(scale)))
    s = np.float32(1.0)
    for l in range(nlevels):
        sizes.append((int(np.rint(np.float32(w) * s)), int(np.rint(np.float32(h) * s))))
        s = np.float32(s * invf)
    return sizes


def algorithmic_bytes(w, h, nfeatures):
    """Per-frame algorithmic bytes per stage."""
    sz = level_sizes(w, h)
    px = [a * b for a, b in sz]
    return {
        "pyr0": px[0] + px[0],                               # read image, write level 0
        "resize": sum(px[l - 1] + px[l] for l in range(1, 8)),
        "fast": sum(px),                                     # one read of every level
        "blur": 2 * sum(px),                                 # read + write
        "describe": nfeatures * (512 + 700 + 60),            # samples, IC patch, outputs
        "retain": 0, "match": 0,
    }


def cpu_baseline(frames, nfeatures, budget_s):
    """Oracle (C++ restatement, 1 core) on a bounded sample of the workload."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    L = oracle_lib.load()
    ex = oracle_lib.RefExtractor(nfeatures)
    h, w = frames.shape[1:]
    t0 = time.perf_counter()
    n = 0
    prev = None
    while time.perf_counter() - t0 < budget_s and n < len(frames) * 4:
        k, d = ex(frames[n % len(frames)])
        if prev is not None:
            F1 = ox.frame_view(prev[0], prev[1], w, h)
            F2 = ox.frame_view(k, d, w, h)
            pm = np.stack([prev[0]["x"], prev[0]["y"]], 1).astype(np.float32).copy()
            m = np.zeros(len(prev[0]), np.int32)
            nm = ctypes.c_int()
            L.orbx_ref_search_for_initialization(ctypes.byref(F1), ctypes.byref(F2), oracle_lib.ptr(pm),
                                                 oracle_lib.ptr(m), 100, 0.9, 1, ctypes.byref(nm))
        prev = (k, d)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{n} frames of the same sequence, extract + SearchForInitialization, "
                      f"oracle/liborbx_ref.so (g++ -O3), 1 thread, {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="frames per step per GPU")
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args()

    world, rank, local = odist.env()
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl")
        dist = tdist

    wl = WORKLOADS[args.workload]
    w, h, nf, B = wl["w"], wl["h"], wl["nfeatures"], args.batch
    frames = synth.sequence(w, h, B, seed=odist.shard_seed(2000, rank))
    ctx = ox.Context(nfeatures=nf, max_w=w, max_h=h, slots=B, device=local if world > 1 else 0)
    ctx.upload(frames)

    def step():
        ctx.extract(0, B)
        ctx.match_prev(0, B, B, window=100, nnratio=0.9, check_ori=True)

    for _ in range(args.warmup):
        step()
    ctx.sync()

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    ctx.timing(True)
    barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    kernels = {}
    for name in ["pyr0", "resize", "fast", "retain", "blur", "describe", "match"]:
        n, avg, tot = ctx.kernel_time(name)
        kernels[name] = {"launches": n, "avg_ms": avg, "total_ms": tot}
    ctx.timing(False)

    # sanity: the last batch produced features and matches
    k0, _ = ctx.features(B - 1)
    _, nm = ctx.matches(B - 1)
    stats = np.array([elapsed, B * args.steps, len(k0), nm], dtype=np.float64)
    allst = odist.gather_stats(stats, dist, device="cuda")
    value, elapsed, _ = odist.job_rate(allst)

    if rank == 0:
        ab = algorithmic_bytes(w, h, nf)
        dom = max((k for k in kernels if kernels[k]["launches"]), key=lambda k: kernels[k]["total_ms"])
        per_launch = ab[dom] * B / max(1, kernels[dom]["launches"] // args.steps)
        avg_s = kernels[dom]["avg_ms"] / 1e3
        achieved = per_launch / avg_s / 1e9 if avg_s > 0 and per_launch > 0 else 0.0
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None, "kernel": dom,
                "algorithmic_bytes_per_launch": per_launch, "avg_launch_ms": kernels[dom]["avg_ms"]}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(frames, nf, args.cpu_budget)
        out = {
            "metric": "frames/sec ORB extract+match (640x480, 1000 kp)" if args.workload == "c2"
            else "pairs/sec ORB extract+match (1920x1080, 2000 kp)",
            "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (orb_slam_amd/synth.py sequence, seed 2000+rank)",
            "config": {"workload": wl["desc"], "frames_per_step_per_gpu": B, "nfeatures": nf,
                       "image": f"{w}x{h}", "parallelism": f"dp{world} (one sequence per GPU)"},
            "roofline": roof, "cpu_baseline": cpu,
            "check": {"last_frame_keypoints": int(stats[2]), "last_frame_matches": int(stats[3])},
        }
        if args.verbose:
            out["kernels"] = kernels
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
