"""Local BA kernel phase breakdown (diagnostic build): s_memtime cycles of
block 0 per phase, summed over a c5-sized batch solve.
Build: python -m orb_slam_amd.build -DORBX_LBA_PROFILE --out=orb_slam_amd/liborbx_lbaprof.so
Run:   ORBX_LIBRARY=orb_slam_amd/liborbx_lbaprof.so python3 tools/lba_phases.py"""
import ctypes
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import synth_ba as sb  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 64
uniq = [sb.make_problem(n_kf=20, n_points=2000, seed=5000 + i) for i in range(8)]
cps = [sb.to_ctypes(uniq[i % 8]) for i in range(P)]
arr = (sb.BAProblem * P)(*[c[0] for c in cps])
es = [np.zeros(c[0].n_edges, np.uint8) for c in cps]
pb = [np.zeros(c[0].n_points, np.uint8) for c in cps]
esp = (ctypes.c_void_p * P)(*[e.ctypes.data for e in es])
pbp = (ctypes.c_void_p * P)(*[b.ctypes.data for b in pb])
ctx = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
L = ox.lib()
L.orbx_debug_lba_prof.argtypes = [ctypes.c_void_p]
before = (ctypes.c_ulonglong * 32)()
L.orbx_debug_lba_prof(before)
st = (sb.BAStats * P)()
assert L.orbx_lba_solve_batch(ctx.handle, P, arr, 5, 10, None, esp, pbp, st) == 0
after = (ctypes.c_ulonglong * 32)()
L.orbx_debug_lba_prof(after)
d = [a - b for a, b in zip(after, before)]
names = {6: "errors (first iteration)", 7: "linearize", 1: "S init", 2: "Schur complement", 3: "dense LLT",
         4: "substitution", 8: "back-subst + update + errors"}
tot = sum(d[k] for k in names)
for k, nm in names.items():
    print(f"{nm:28s} {d[k]:14d} ({100.0 * d[k] / max(tot, 1):5.1f} %)")
# k_lba_build (the first optimize() call's structures), block 0
build = {9: "build: flags", 10: "build: rank ids", 11: "build: count atomics", 12: "build: offsets + scatter",
         13: "build: per-point sort", 14: "build: records", 15: "build: per-pose lists"}
btot = sum(d[k] for k in build)
for k, nm in build.items():
    print(f"{nm:28s} {d[k]:14d} ({100.0 * d[k] / max(btot, 1):5.1f} % of the build)")
# k_lba_split (a batch of one over several workgroups), workgroup 0
split = {16: "split: errors + linearize", 17: "split: barrier + maxima", 18: "split: Schur (LDS)",
         19: "split: slab + barrier", 20: "split: slice sums + barrier", 21: "split: convert", 22: "split: LLT + solve",
         23: "split: back-subst + errors", 24: "split: barrier", 25: "split: sums + decision"}
stot = sum(d[k] for k in split)
for k, nm in split.items():
    if stot:
        print(f"{nm:28s} {d[k]:14d} ({100.0 * d[k] / stot:5.1f} %)")
print(f"{'LLT: panel steps':28s} {d[26]:14d}")
print(f"{'LLT: trailing steps':28s} {d[27]:14d}")
print("iterations", list(st[0].iterations), "trials", list(st[0].levenberg_trials), "n_edges", cps[0][0].n_edges)
