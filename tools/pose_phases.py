"""Phase times of the exact one-frame PoseOptimization kernel
(k_pose_exact_wide) from the ORBX_POSE_PROFILE build: round-start builds,
solves, trial passes, classification (wall clock of block 0, thread 0).

usage: python tools/pose_phases.py [--n N]   (builds build_orbx_pose_profile/ on first use)
"""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
LIBP = ROOT / "orb_slam_amd" / "liborbx_pose_profile.so"
os.environ["ORBX_LIBRARY"] = str(LIBP)
import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import synth_pose as sp  # noqa: E402

if not LIBP.exists():
    from orb_slam_amd import build as b
    b.build(defines=("ORBX_POSE_PROFILE",), lib=LIBP)
args = sys.argv[1:]
n = int(args[args.index("--n") + 1]) if "--n" in args else 50
L = ox.lib()
L.orbx_debug_pose_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
ctx = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
assert L.orbx_pose_set_exact(ctx.handle, 1) == 0
p, arrs = sp.to_ctypes(sp.make_frame(n_kp=1000, seed=7))
w = sp.PoseFrame.from_buffer_copy(p)
ni = ctypes.c_int()
st = sp.PoseStats()
buf = (ctypes.c_ulonglong * 8)()
for i in range(n + 5):
    if i == 5:
        L.orbx_debug_pose_prof(buf, 1)
    ctypes.memmove(ctypes.addressof(w), ctypes.addressof(p), ctypes.sizeof(w))
    assert L.orbx_pose_optimization(ctx.handle, ctypes.byref(w), ctypes.byref(ni), ctypes.byref(st)) == 0
L.orbx_debug_pose_prof(buf, 0)
v = np.array(list(buf), np.float64)
us = v[:5] / 100.0 / n          # 100 MHz ticks -> us per call
print(f"ldlt part of solves: {v[7] / 100.0 / n:.1f} us per call")
print(f"edges {int(np.count_nonzero(arrs['has_mp']))} iterations {list(st.iterations)} trials {list(st.levenberg_trials)}")
print(f"per call: kernel {us[4]:.1f} us = builds {us[0]:.1f} ({v[5] / n:.1f}x) + solves {us[1]:.1f} + trials "
      f"{us[2]:.1f} ({v[6] / n:.1f}x) + classify {us[3]:.1f} + rest {us[4] - us[:4].sum():.1f}")
ctx.close()
