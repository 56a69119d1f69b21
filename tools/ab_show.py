"""Print the headline of a tools/gpu_fast_ab.sh result directory."""
import json
import sys
from pathlib import Path

d = Path(sys.argv[1])
c2 = json.loads(open(d / "c2.json").read())
print("c2", c2["value"], "ms/step", c2["ms_per_step"], "fast serial avg", c2["roofline"]["avg_launch_ms"])
s = json.loads(open(d / "c2_serial.json").read())
k = s["kernels"]["serial"]
steps = s["kernels"]["serial_steps"]
B = s["config"]["frames_per_step_per_gpu"]
print("serial us per 256 frames:", {n: round(1e3 * v["total_ms"] / steps * 256 / B, 1) for n, v in k.items()})
p = d / "fast_phases.txt"
if p.exists():
    print(p.read_text())
