"""llt_solve alone (diagnostic build): cycles per factorisation + solve of a
random SPD system of n = 6 nb, and the LLT phase split of the profile marks.
Build: python -m orb_slam_amd.build -DORBX_LBA_PROFILE --out=orb_slam_amd/liborbx_lbaprof.so
Run:   ORBX_LIBRARY=orb_slam_amd/liborbx_lbaprof.so python3 tools/llt_bench.py [nb ...]"""
import ctypes
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import orb_slam_amd as ox  # noqa: E402

L = ox.lib()
L.orbx_debug_llt_bench.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
L.orbx_debug_lba_prof.argtypes = [ctypes.c_void_p]
L.orbx_debug_llt_waves.argtypes = [ctypes.c_void_p]
import time
reps = 50
for nb in [int(a) for a in sys.argv[1:]] or [20]:
    mode = 0
    n = 6 * nb
    rng = np.random.default_rng(nb)
    A = rng.standard_normal((n, n))
    H = A @ A.T + n * np.eye(n)
    b = rng.standard_normal(n)
    packed = np.concatenate([H[i, :i + 1] for i in range(n)] + [b])
    x = np.zeros(n)
    cyc = ctypes.c_ulonglong(0)
    before = (ctypes.c_ulonglong * 32)()
    L.orbx_debug_lba_prof(before)
    wb = (ctypes.c_ulonglong * 32)()
    L.orbx_debug_llt_waves(wb)
    assert L.orbx_debug_llt_bench(packed.ctypes.data, n, reps, x.ctypes.data, ctypes.byref(cyc), mode) == 0
    after = (ctypes.c_ulonglong * 32)()
    L.orbx_debug_lba_prof(after)
    wa = (ctypes.c_ulonglong * 32)()
    L.orbx_debug_llt_waves(wa)
    w = np.array([(a - bb) // reps for a, bb in zip(wa, wb)]).reshape(8, 4)
    wall = []
    for rr in (reps, 10 * reps):   # wall-clock calibration of the cycle counter
        t0 = time.perf_counter()
        L.orbx_debug_llt_bench(packed.ctypes.data, n, rr, x.ctypes.data, ctypes.byref(ctypes.c_ulonglong(0)), mode)
        wall.append(time.perf_counter() - t0)
    us = (wall[1] - wall[0]) / (9 * reps) * 1e6
    d = [(a - bb) // reps for a, bb in zip(after, before)]
    err = np.abs(x - np.linalg.solve(H, b)).max()
    print(f"nb {nb:3d} n {n:4d}: {cyc.value / reps:10.0f} cycles per solve; panel {d[26]} trailing {d[27]} "
          f"substitution {d[4]}; max |x - x_np| {err:.2e}; {us:.1f} us per solve "
          f"({cyc.value / reps / us / 1e3:.2f} GHz counter)")
    if w.any():
        for wv in range(8):
            print(f"   wave {wv}: panel work {w[wv, 0]:7d} wait {w[wv, 1]:7d}  trailing work {w[wv, 2]:7d} wait {w[wv, 3]:7d}")

# latency probes (one wave... the whole workgroup runs them): cycles per dependent op
n = 120
v = np.concatenate([np.full(n, 1.0000001), np.full(n, 0.9999999)] + [np.zeros(n * (n + 1) // 2)])
x = np.zeros(n)
x120 = x
for mode, name in ((2, "f64 mul"), (3, "rsqrt_nr"), (5, "workgroup barrier"), (6, "LDS load")):
    cyc = ctypes.c_ulonglong(0)
    L.orbx_debug_llt_bench(v.ctypes.data, n, 1, x.ctypes.data, ctypes.byref(cyc), mode)
    print(f"{name}: {cyc.value / 1000:.1f} counter ticks per dependent op")
# v_rsq_f64 accuracy
n = 120
x = np.zeros(n)
rng = np.random.default_rng(7)
xs = np.exp(rng.uniform(-30, 30, n))
buf = np.concatenate([xs, np.zeros(n * (n + 1) // 2)])
L.orbx_debug_llt_bench(buf.ctypes.data, n, 1, x.ctypes.data, ctypes.byref(ctypes.c_ulonglong(0)), 4)
ref = 1.0 / np.sqrt(xs)
ulp = np.abs(x - ref) / np.spacing(ref)
print(f"v_rsq_f64: max error {ulp.max():.1f} ulp, median {np.median(ulp):.1f} ulp")
