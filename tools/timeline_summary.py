"""Summarise a rocprofv3 --kernel-trace of the c2 bench (tools/gpu_c2_modes.sh):
per kernel class, busy time (union of its dispatch intervals), and the time
during which each class runs alone.  usage: timeline_summary.py run_kernel_trace.csv [steps]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = []
for r in rows:
    n = r["Kernel_Name"]
    m = re.search(r"k_(\w+?)(<|\(|$)", n)
    k = m.group(1) if m else n[:20]
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
ev.sort()
# last 4 steps' window: drop the first third of the trace (setup/warmup)
t0 = ev[len(ev) // 3][0]
t1 = ev[-1][1]
ev = [e for e in ev if e[0] >= t0]
span = t1 - t0
busy = defaultdict(int)
alone = defaultdict(int)
pts = sorted({e[0] for e in ev} | {e[1] for e in ev})
for a, b in zip(pts, pts[1:]):
    act = {e[2] for e in ev if e[0] < b and e[1] > a}
    for k in act:
        busy[k] += b - a
    if len(act) == 1:
        alone[next(iter(act))] += b - a
    if not act:
        alone["<idle>"] += b - a
print(f"window {span / 1e3:.1f} us")
for k in sorted(busy, key=lambda k: -busy[k]):
    print(f"{k:20s} busy {busy[k] / 1e3:9.1f} us ({100 * busy[k] / span:5.1f} %)  alone {alone[k] / 1e3:8.1f} us")
print(f"{'<idle>':20s} {alone['<idle>'] / 1e3:9.1f} us")
