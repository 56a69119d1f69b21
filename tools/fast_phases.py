"""FAST kernel phase breakdown (diagnostic build): per-phase cycles summed
over workgroups (s_memtime stamps of thread 0), compass survivors and units.
Build: python -m orb_slam_amd.build -DORBX_FAST_PROFILE --out=orb_slam_amd/liborbx_fastprof.so
Run:   ORBX_LIBRARY=orb_slam_amd/liborbx_fastprof.so python3 tools/fast_phases.py [W H nfeatures frames]"""
import ctypes
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import synth  # noqa: E402

W, H, NF, B = (int(v) for v in sys.argv[1:5]) if len(sys.argv) > 4 else (640, 480, 1000, 256)
ctx = ox.Context(nfeatures=NF, max_w=W, max_h=H, slots=B)
ctx.upload(synth.sequence(W, H, B, seed=2000))
ctx.set_split(False)
ctx.extract(0, B)
ctx.sync()
L = ox.lib()
buf = (ctypes.c_ulonglong * 16)()
L.orbx_debug_fast_prof.argtypes = [ctypes.c_void_p]
before = list(buf) if L.orbx_debug_fast_prof(buf) == 0 else None
ctx.extract(0, B)
ctx.sync()
after = (ctypes.c_ulonglong * 16)()
L.orbx_debug_fast_prof(after)
d = [a - b for a, b in zip(after, before)]
names = {7: "start..tile load (geometry)", 5: "tile loads + LDS stores", 6: "clear S'/nz",
         0: "first barrier wait", 1: "score@th", 2: "nms@th", 3: "fallback(score+nms@7)", 4: "compact+store",
         8: "fallback cells", 9: "cells", 10: "survivors@th", 11: "survivors@7", 12: "unit batches"}
stamped = (0, 1, 2, 3, 4, 5, 6, 7)
tot = sum(d[k] for k in stamped)
for k, n in names.items():
    v = d[k]
    extra = f" ({100.0 * v / tot:.1f} % of stamped cycles)" if k in stamped and tot else ""
    print(f"{n:24s} {v:16d}{extra}")
