"""Where a single-pair SearchForInitialization call (k_search_init_one) spends
its cycles: the ORBX_MATCH_PROFILE build's wave-0 stamps of block 0.

  python -m orb_slam_amd.build -DORBX_MATCH_PROFILE --out=orb_slam_amd/liborbx_matchprof.so
  ORBX_LIBRARY=orb_slam_amd/liborbx_matchprof.so python3 tools/sfi_phases.py [calls]"""
import ctypes
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))

import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import synth  # noqa: E402
import oracle_lib  # noqa: E402

NAMES = {0: "stage F2 + F1 tables", 4: "count pass (group 0)", 5: "count barrier (group 0)",
         6: "fill pass (group 0)", 1: "scan + fill (all groups)", 7: "greedy replay (wave 0)",
         2: "end of groups", 3: "rotation check + output"}


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    w, h, nf = 640, 480, 1000
    frames = synth.sequence(w, h, 8, seed=2000)
    rex = oracle_lib.RefExtractor(nf)
    feats = [rex(np.ascontiguousarray(f)) for f in frames]
    views = [ox.frame_view(k, d, w, h) for k, d in feats]
    L = ox.lib()
    prof_fn = getattr(L, "orbx_debug_search_prof", None)   # absent from the product build: timing only
    if prof_fn is not None:
        prof_fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ctx = ox.Context(nfeatures=nf, max_w=w, max_h=h, slots=1)
    m12 = np.zeros(nf, np.int32)
    pm = np.zeros((nf, 2), np.float32)
    nm = ctypes.c_int()
    prof = np.zeros(12, np.uint64)
    ts = []
    for c in range(calls + 20):
        i = c % 7
        k = feats[i][0]
        pm[:len(k)] = np.stack([k["x"], k["y"]], 1)
        if c == 20 and prof_fn is not None:
            prof_fn(prof.ctypes.data, 1)
        t0 = time.perf_counter()
        r = L.orbx_search_for_initialization(ctx.handle, ctypes.byref(views[i]), ctypes.byref(views[i + 1]),
                                             pm.ctypes.data, m12.ctypes.data, 100, 0.9, 1, ctypes.byref(nm))
        ts.append(time.perf_counter() - t0)
        assert r == 0, r
    print(f"median call {1e3 * np.median(ts[20:]):.3f} ms ({ox.LIB_PATH})")
    if prof_fn is None:
        ctx.close()
        return
    prof_fn(prof.ctypes.data, 0)
    tot = int(prof[:8].sum())
    print("per call:")
    for k in (0, 4, 5, 6, 1, 7, 2, 3):
        v = int(prof[k]) / calls
        print(f"  {NAMES[k]:28s} {v:10.0f} cycles ({100 * int(prof[k]) / max(tot, 1):5.1f} %)")
    print(f"  replay per call: {int(prof[8]) / calls:.1f} queries with candidates, {int(prof[9]) / calls:.1f} "
          f"full passes, {int(prof[10]) / calls:.1f} accepted")
    ctx.close()


if __name__ == "__main__":
    main()
