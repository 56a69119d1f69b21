"""Summary of tools/gpu_pmc_libs.sh: per library, the named kernels' counters
and serialised time.  usage: python tools/pmc_libs_summary.py gpurun_out/<tag> [kernel substrings]"""
import collections
import csv
import glob
import sys
from pathlib import Path

d = Path(sys.argv[1])
keys = sys.argv[2:] or ["fast"]
for p in sorted(x for x in d.glob("p_*") if x.is_dir()):
    n = p.name[2:]
    g = glob.glob(str(p / "**" / "*counter_collection.csv"), recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(g[0])):
        agg[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
    t = {}
    s = d / f"s_{n}" / "run_kernel_stats.csv"
    if s.exists():
        t = {r["Name"][:40]: float(r["AverageNs"]) / 1000 for r in csv.DictReader(open(s))}
    for k, v in agg.items():
        if any(x in k for x in keys):
            print(f"{n:16s} {k[:30]:30s} {t.get(k, 0):7.1f}us " + " ".join(
                f"{c.replace('SQ_', '')}={x:.3e}" for c, x in sorted(v.items())))
