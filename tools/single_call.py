"""Single-call workloads for kernel traces of the drop-in path (run from the
repo root on the GPU box, under `rocprofv3 --kernel-trace --memory-copy-trace
--stats`): N calls each of

  extract   orbx_extract on one 640x480 frame (graph launch mode, then stream
            launches): ORBextractor::operator() as Frame::Frame calls it
  sfi       orbx_search_for_initialization on two host frame views
  pose      orbx_pose_optimization on one frame
  lba       orbx_lba_solve on one 20 KF x 2000 MP problem
  search    the Tracking searches on host frame views
  track     orbx_track_frame: one whole Tracking frame (image in), then the
            chain alone (slot already extracted)

usage: python tools/single_call.py [extract] [sfi] [pose] [lba] [search] [track] [--n N] [--lbawg g,...] [--coop c,...]
"""
import ctypes
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import synth  # noqa: E402

args = sys.argv[1:]
n = int(args[args.index("--n") + 1]) if "--n" in args else 100
what = [a for a in args if a in ("extract", "sfi", "pose", "lba", "search", "track")] or ["extract"]
lbawg = [int(v) for v in args[args.index("--lbawg") + 1].split(",")] if "--lbawg" in args else [0]
# k_lba_split launch: -1 the device's choice, 0 plain, 1 cooperative (orbx_debug_lba_split)
coop = [int(v) for v in args[args.index("--coop") + 1].split(",")] if "--coop" in args else [-1]
L = ox.lib()


def med(fn, k):
    t = []
    for i in range(k):
        t0 = time.perf_counter()
        fn(i)
        t.append(time.perf_counter() - t0)
    return 1e3 * float(np.median(t))


if "extract" in what or "sfi" in what:
    frames = synth.sequence(640, 480, 16, seed=2000)
    ctx = ox.Context(nfeatures=1000, max_w=640, max_h=480, slots=1)
    kps = np.zeros(1000, ox.KEYPOINT)
    desc = np.zeros((1000, 32), np.uint8)
    nk = ctypes.c_int()

    def ext(i):
        assert L.orbx_extract(ctx.handle, frames[i % 16].ctypes.data, 640, 480, 640, kps.ctypes.data,
                              desc.ctypes.data, 1000, ctypes.byref(nk)) == 0

    if "extract" in what:
        for mode in (1, 0):
            ctx.set_launch_mode(mode)
            print(f"extract launch mode {mode}: {med(ext, n):.4f} ms median", flush=True)
        ctx.set_launch_mode(1)
    if "sfi" in what:
        feats = [ctx(frames[i]) for i in range(2)]
        F1 = ox.frame_view(*feats[0], 640, 480)
        F2 = ox.frame_view(*feats[1], 640, 480)
        k1 = feats[0][0]
        pm = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
        m = np.zeros(len(k1), np.int32)
        nm = ctypes.c_int()

        def sfi(i):
            pm[:] = np.stack([k1["x"], k1["y"]], 1)
            assert L.orbx_search_for_initialization(ctx.handle, ctypes.byref(F1), ctypes.byref(F2), pm.ctypes.data,
                                                    m.ctypes.data, 100, 0.9, 1, ctypes.byref(nm)) == 0

        print(f"sfi: {med(sfi, n):.4f} ms median", flush=True)
    ctx.close()

if "search" in what:
    # the per-frame Tracking searches (host-pointer calls) against the CPU port
    from oracle_lib import RefExtractor, load, ptr
    W, H = 640, 480
    CAM = np.array([500.0, 500.0, 320.0, 240.0], np.float32)
    fr = synth.sequence(W, H, 3, seed=77)
    ex = RefExtractor(1000)
    (kl, dl), (kc, dc) = ex(fr[1]), ex(fr[2])
    C, Lv = ox.frame_view(kc, dc, W, H), ox.frame_view(kl, dl, W, H)
    rng = np.random.default_rng(15)
    z = rng.uniform(2, 6, len(kl)).astype(np.float32)
    xyz = np.ascontiguousarray(np.stack([(kl["x"] - CAM[2]) / CAM[0] * z, (kl["y"] - CAM[3]) / CAM[1] * z, z],
                                        1).astype(np.float32))
    valid = (rng.random(len(kl)) < 0.85).astype(np.uint8)
    asg = np.zeros(len(kc), np.uint8)
    c_, s_ = np.cos(0.002), np.sin(0.002)
    T = np.array([[c_, 0, s_, -0.008], [0, 1, 0, -0.004], [-s_, 0, c_, 0]], np.float32).reshape(-1).copy()
    m = np.zeros(len(kc), np.int32)
    nm = ctypes.c_int()
    R = load()
    ctx = ox.Context(nfeatures=1000, max_w=W, max_h=H, slots=1)
    calls = {
        "motion th15": (lambda i: L.orbx_search_by_projection_motion(ctx.handle, ctypes.byref(C), ctypes.byref(Lv),
                                                                    ptr(xyz), ptr(valid), ptr(asg), ptr(T), ptr(CAM),
                                                                    15.0, 1, ptr(m), ctypes.byref(nm)),
                        lambda i: R.orbx_ref_search_by_projection_motion(ctypes.byref(C), ctypes.byref(Lv), ptr(xyz),
                                                                        ptr(valid), ptr(asg), ptr(T), ptr(CAM), 15.0, 1,
                                                                        ptr(m), ctypes.byref(nm))),
        "window 200": (lambda i: L.orbx_window_search(ctx.handle, ctypes.byref(Lv), ctypes.byref(C), ptr(valid), 200,
                                                      0, -1, 0.9, 1, ptr(m), ctypes.byref(nm)),
                       lambda i: R.orbx_ref_window_search(ctypes.byref(Lv), ctypes.byref(C), ptr(valid), 200, 0, -1,
                                                          0.9, 1, ptr(m), ctypes.byref(nm))),
        "pair 15": (lambda i: L.orbx_search_by_projection_pair(ctx.handle, ctypes.byref(Lv), ctypes.byref(C),
                                                               ptr(xyz), ptr(valid), ptr(asg), ptr(T), ptr(CAM), 15,
                                                               0.9, ptr(m), ctypes.byref(nm)),
                    lambda i: R.orbx_ref_search_by_projection_pair(ctypes.byref(Lv), ctypes.byref(C), ptr(xyz),
                                                                   ptr(valid), ptr(asg), ptr(T), ptr(CAM), 15, 0.9,
                                                                   ptr(m), ctypes.byref(nm))),
    }
    dbg = (ctypes.c_ulonglong * 2)()
    L.orbx_debug_area_rounds.argtypes = [ctypes.c_void_p]
    for name, (g, c) in calls.items():
        L.orbx_debug_area_rounds(dbg)
        r0 = list(dbg)
        tg = med(g, n)
        L.orbx_debug_area_rounds(dbg)
        print(f"search {name}: gpu {tg:.4f} ms, cpu port {med(c, max(5, n // 4)):.4f} ms median; "
              f"replay rounds {(dbg[0] - r0[0]) / n:.2f} per call, sequential fallbacks {dbg[1] - r0[1]} of {n}",
              flush=True)
    ctx.close()

if "track" in what:
    import track_data as td
    W, H = 640, 480
    ctx = ox.Context(nfeatures=1000, max_w=W, max_h=H, slots=3)
    last_img, cur_img = td.images(W, H, 6, 11)
    ctx.upload(last_img, 0)
    ctx.extract(0, 1)
    ctx.sync()
    kl, dl = ctx.features(0)
    scene = td.make_scene(kl, dl, 11)
    Tp = td.pose_x(7.5 * td.DEPTH / float(td.CAM[0]))
    qi, ki = td.query(scene, Tp, slot=1, image=cur_img, last_slot=0)
    qs, ks = td.query(scene, Tp, slot=1, last_slot=0)
    for exact in (0, 1):
        assert L.orbx_pose_set_exact(ctx.handle, exact) == 0
        ti = med(lambda i: L.orbx_track_frame(ctx.handle, ctypes.byref(qi)), n)
        tc = med(lambda i: L.orbx_track_frame(ctx.handle, ctypes.byref(qs)), n)
        r = td.result(qs, ks)
        print(f"track (exact sums {exact}): image in {ti:.4f} ms, chain only {tc:.4f} ms median; status "
              f"{r['status']} motion {r['n_motion']} in view {r['n_in_view']} local {r['n_local']} "
              f"inliers {r['n_inliers']}", flush=True)
    assert L.orbx_pose_set_exact(ctx.handle, 1) == 0
    qp, kp = td.query(scene, td.pose_x(0.0), slot=1, last_slot=0, mode=1)
    tp = med(lambda i: L.orbx_track_frame(ctx.handle, ctypes.byref(qp)), n)
    r = td.result(qp, kp)
    print(f"track previous frame (mode 1): chain only {tp:.4f} ms median; status {r['status']} window "
          f"{r['n_motion']} pair {r['n_pair']} local {r['n_local']} inliers {r['n_inliers']}", flush=True)
    ctx.close()

if "pose" in what:
    from orb_slam_amd import synth_pose as sp
    ctx = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
    p, arrs = sp.to_ctypes(sp.make_frame(n_kp=1000, seed=7))
    w = sp.PoseFrame.from_buffer_copy(p)
    ni = ctypes.c_int()

    def pose(i):
        ctypes.memmove(ctypes.addressof(w), ctypes.addressof(p), ctypes.sizeof(w))
        assert L.orbx_pose_optimization(ctx.handle, ctypes.byref(w), ctypes.byref(ni), None) == 0

    print(f"pose: {med(pose, n):.4f} ms median", flush=True)
    ctx.close()

if "lba" in what:
    from orb_slam_amd import synth_ba as sb
    ctx = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
    pr = sb.make_problem(n_kf=20, n_points=2000, seed=5)
    p, arrs = sb.to_ctypes(pr)
    es = np.zeros(p.n_edges, np.uint8)
    pb = np.zeros(p.n_points, np.uint8)
    st = sb.BAStats()

    def lba(i):
        np.copyto(arrs["pose_q"], pr["pose_q"])
        np.copyto(arrs["pose_t"], pr["pose_t"])
        np.copyto(arrs["points"], pr["points"])
        assert L.orbx_lba_solve(ctx.handle, ctypes.byref(p), 5, 10, None, es.ctypes.data, pb.ctypes.data,
                                ctypes.byref(st)) == 0

    for cp in coop:
        assert L.orbx_debug_lba_split(ctx.handle, -1, -1, -1, cp) == 0
        for wg in lbawg:
            assert L.orbx_lba_set_workgroups(ctx.handle, wg) == 0
            t = med(lba, max(5, n // 10))
            print(f"lba coop {cp} workgroups {wg} (ran {L.orbx_lba_last_workgroups(ctx.handle)}): {t:.4f} ms median",
                  flush=True)
    ctx.close()
print("ok")
