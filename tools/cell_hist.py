"""Distribution of per-cell FAST list lengths at C2 (640x480, 1000 kp) on the
bench's synthetic sequence (run on the GPU box)."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, "/root/repo")
import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import synth  # noqa: E402

B = 16
ctx = ox.Context(nfeatures=1000, max_w=640, max_h=480, slots=B)
ctx.upload(synth.sequence(640, 480, B, seed=2000))
ctx.extract(0, B)
ctx.sync()
L = ox.lib()
L.orbx_debug_cells.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
counts, levels = [], []
for s in range(B):
    buf = np.zeros(9 * 4096, np.int32)
    n = L.orbx_debug_cells(ctx.handle, s, buf.ctypes.data, buf.size)
    c = buf[:9 * n].reshape(n, 9)
    counts.append(c[:, 7])
    levels.append(c[:, 0])
counts, levels = np.concatenate(counts), np.concatenate(levels)
for lo, hi in [(0, 8), (9, 64), (65, 128), (129, 256), (257, 512), (513, 10 ** 6)]:
    sel = (counts >= lo) & (counts <= hi)
    print(f"n in [{lo},{hi}]: {sel.mean() * 100:5.1f} % of cells, {counts[sel].sum() / counts.sum() * 100:5.1f} % of entries")
for l in range(8):
    print("level", l, "median n", int(np.median(counts[levels == l])), "max", counts[levels == l].max())
