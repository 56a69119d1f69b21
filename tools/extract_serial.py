"""Serialised extraction + matching (pipeline split off), four times: the
workload behind the per-kernel `rocprofv3 --kernel-trace` and `--pmc SQ_*`
tables in profiles/ (run from the repo root on the GPU box).

  (default)  256 frames of 640x480, 1000 kp, SearchForInitialization (c2)
  --hd       32 frames of 1920x1080, 2000 kp, brute-force matching (c3)
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import synth  # noqa: E402

hd = "--hd" in sys.argv[1:]
W, H, N, B = (1920, 1080, 2000, 32) if hd else (640, 480, 1000, 256)
ctx = ox.Context(nfeatures=N, max_w=W, max_h=H, slots=B)
ctx.upload(synth.sequence(W, H, B, seed=2000))
ctx.set_split(False)
for _ in range(4):
    ctx.extract(0, B)
    if hd:
        ctx.match_bf_prev(0, B, B)
    else:
        ctx.match_prev(0, B, B)
ctx.sync()
print("ok")
