"""Fused pyramid kernel phase breakdown (diagnostic build): per wave, cycles
summed over the workgroups in setup / level-0 items / resize / blur / barrier
wait, with the wave's jobs from the plan.
Build: python3 -c "from orb_slam_amd import build; build.build(defines=('ORBX_PYR_PROFILE',), lib='orb_slam_amd/liborbx_pyrprof.so')"
Run:   ORBX_LIBRARY=orb_slam_amd/liborbx_pyrprof.so python3 tools/pyr_phases.py [W H nfeatures frames]"""
import ctypes
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import synth  # noqa: E402

W, H, NF, B = (int(v) for v in sys.argv[1:5]) if len(sys.argv) > 4 else (640, 480, 1000, 256)
ctx = ox.Context(nfeatures=NF, max_w=W, max_h=H, slots=B)
ctx.set_pyramid_mode(1)
ctx.upload(synth.sequence(W, H, B, seed=2000))
ctx.set_split(False)
ctx.extract(0, B)
ctx.sync()
print("fused:", ctx.pyramid_fused())
L = ox.lib()
L.orbx_debug_pyr_prof.argtypes = [ctypes.c_void_p]
before = (ctypes.c_ulonglong * 80)()
L.orbx_debug_pyr_prof(before)
ctx.extract(0, B)
ctx.sync()
after = (ctypes.c_ulonglong * 80)()
L.orbx_debug_pyr_prof(after)
d = [(a - b) / B for a, b in zip(after, before)]
print(f"{'wave':>4} {'setup':>9} {'l0':>9} {'resize':>9} {'blur':>9} {'barrier':>9}   (cycles per workgroup)")
for w in range(16):
    r = d[5 * w:5 * w + 5]
    print(f"{w:4d} {r[4]:9.0f} {r[0]:9.0f} {r[1]:9.0f} {r[2]:9.0f} {r[3]:9.0f}")
