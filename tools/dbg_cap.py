"""Diagnose a configuration the product refuses: which device error flag,
which level / cell (run on the GPU box from the repo root)."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, "/root/repo")
sys.path.insert(0, "/root/repo/tests")
import orb_slam_amd as ox  # noqa: E402
from test_extract_gpu import make  # noqa: E402

# usage: dbg_cap.py [w h nf scale nlevels fastTh score kind seed]
a = sys.argv[1:]
if a:
    w, h, nf, sc, nl, fth, score, kind, seed = (int(a[0]), int(a[1]), int(a[2]), float(np.float32(float(a[3]))),
                                                int(a[4]), int(a[5]), int(a[6]), a[7], int(a[8]))
else:
    w, h, nf, sc, nl, fth, score, kind, seed = 237, 373, 1518, float(np.float32(1.3333345651626587)), 10, 39, 1, "texture", 3
img = make(kind, w, h, seed)
ctx = ox.Context(nfeatures=nf, scale_factor=sc, nlevels=nl, fast_th=fth, score_type=score, max_w=w, max_h=h, slots=1)
L = ox.lib()
L.orbx_debug_error_flags.argtypes = [ctypes.c_void_p]
ctx.upload(img)
ctx.extract(0, 1)
print("flags", L.orbx_debug_error_flags(ctx.handle))
for lvl in range(nl):
    g = ctx.level(0, lvl)
    print(lvl, g.shape)
L.orbx_debug_cells.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(9 * 4096, np.int32)
n = L.orbx_debug_cells(ctx.handle, 0, buf.ctypes.data, buf.size)
cells = buf[:9 * n].reshape(n, 9)
bad = cells[cells[:, 7] > cells[:, 8]]
print("cells", n, "overflowing", len(bad))
for c in bad[:10]:
    print("level %d i %d j %d ini (%d,%d) h (%d,%d) count %d cap %d" % tuple(c))
