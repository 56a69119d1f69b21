"""Single-frame cascade pyramid (k_pyr_cascade in orbx_extract's graph): band
0's cycles per level and phase, from the -DORBX_CASC_PROFILE build.

  python -m orb_slam_amd.build -DORBX_CASC_PROFILE --out=orb_slam_amd/liborbx_cascprof.so
  ORBX_LIBRARY=orb_slam_amd/liborbx_cascprof.so python3 tools/casc_phases.py [calls]"""
import ctypes
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
frames = synth.sequence(640, 480, 16, seed=2000)
ctx = ox.Context(nfeatures=1000, max_w=640, max_h=480, slots=1)
kps = np.zeros(1000, ox.KEYPOINT)
desc = np.zeros((1000, 32), np.uint8)
nk = ctypes.c_int()
L = ox.lib()
L.orbx_debug_casc_prof.argtypes = [ctypes.c_void_p]


def ext(i):
    assert L.orbx_extract(ctx.handle, frames[i % 16].ctypes.data, 640, 480, 640, kps.ctypes.data, desc.ctypes.data,
                          1000, ctypes.byref(nk)) == 0


for i in range(20):
    ext(i)
before = np.zeros((16, 4), np.uint64)   # kMaxLevels rows
L.orbx_debug_casc_prof(before.ctypes.data)
for i in range(n):
    ext(i)
after = np.zeros((16, 4), np.uint64)
L.orbx_debug_casc_prof(after.ctypes.data)
d = (after - before).astype(np.float64) / n
print("cycles per call, band 0 (load/resize, barrier 1, border + barrier 2, stores):")
for l in range(8):
    print(f"  level {l}: " + "  ".join(f"{v:8.0f}" for v in d[l]) + f"   total {d[l].sum():8.0f}")
print(f"all levels {d.sum():.0f}")
