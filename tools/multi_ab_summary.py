"""Summary of tools/gpu_multi_ab.sh: per library, bench values and the
serialised per-kernel times of the kernels named on the command line.
usage: python tools/multi_ab_summary.py gpurun_out/<tag> [kernel substrings...]"""
import csv
import json
import sys
from pathlib import Path

d = Path(sys.argv[1])
keys = sys.argv[2:] or ["fast", "describe"]
for b in sorted(d.glob("b_*.json")):
    v = [round(json.loads(l)["value"]) for l in b.read_text().splitlines() if l.startswith("{")]
    print(f"{b.stem[2:]:24s} bench {v}")
for s in sorted(d.glob("s_*/run_kernel_stats.csv")):
    for r in csv.DictReader(open(s)):
        if any(k in r["Name"] for k in keys):
            print(f"{s.parent.name[2:]:24s} {r['Name'][:44]:44s} {float(r['AverageNs']) / 1000:8.1f} us")
