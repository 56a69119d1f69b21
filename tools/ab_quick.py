"""Summary of a tools/gpu_ab.sh (+ gpu_fast_diag.sh) directory: bench values of
both libraries, serialised per-kernel times and, when present, SQ counters.
usage: python tools/ab_quick.py gpurun_out/<tag> [kernel substrings...]"""
import collections
import csv
import json
import sys
from pathlib import Path

d = Path(sys.argv[1])
keys = sys.argv[2:] or ["fast"]
t = d / "tests.log"
if t.exists():
    print("tests:", t.read_text().strip().splitlines()[-1])
for f in ("new", "base"):
    p = d / f"{f}.json"
    if p.exists():
        v = [json.loads(l)["value"] for l in p.read_text().splitlines() if l.startswith("{")]
        print(f"{f:5s} bench", [round(x) for x in v])
for f in ("snew", "sbase"):
    p = d / f / "run_kernel_stats.csv"
    if p.exists():
        for r in csv.DictReader(open(p)):
            if any(k in r["Name"] for k in keys):
                print(f"{f:5s} {r['Name'][:48]:48s} {float(r['AverageNs']) / 1000:8.1f} us x{r['Calls']}")
for f in ("sq_new", "sq_base"):
    p = d / f / "run_counter_collection.csv"
    if p.exists():
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(p)):
            agg[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
        for k, v in agg.items():
            if any(x in k for x in keys):
                print(f, k, " ".join(f"{c.replace('SQ_', '')}={x:.3e}" for c, x in sorted(v.items())))
