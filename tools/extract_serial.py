"""Serialised extraction + matching of 256 frames (two-stream split off), four
times: the workload behind the per-kernel `rocprofv3 --kernel-trace` and
`--pmc SQ_*` tables in profiles/ (run from the repo root on the GPU box)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import synth  # noqa: E402

B = 256
ctx = ox.Context(nfeatures=1000, max_w=640, max_h=480, slots=B)
ctx.upload(synth.sequence(640, 480, B, seed=2000))
ctx.set_split(False)
for _ in range(4):
    ctx.extract(0, B)
    ctx.match_prev(0, B, B)
ctx.sync()
print("ok")
