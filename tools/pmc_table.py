"""Per-kernel counters of a rocprofv3 --pmc CSV: the mean per dispatch and the
sum per step.

A kernel launched several times per step (k_pyr_resize_lds: once per level)
has a per-dispatch mean that is a fraction of its cost per step; the per-step
sum is mean x (its dispatches / the anchor kernel's dispatches), the anchor
being a kernel launched once per step (default k_fast_cells; else the kernel
with the fewest dispatches).  --frames N divides the per-step sums by the N
frames (or problems) one anchor dispatch covers.

usage: python tools/pmc_table.py <run_counter_collection.csv> [--anchor NAME] [--frames N]"""
import csv
import sys
from collections import defaultdict

args = sys.argv[1:]
path = args[0]
anchor = args[args.index("--anchor") + 1] if "--anchor" in args else "k_fast_cells"
frames = float(args[args.index("--frames") + 1]) if "--frames" in args else None

acc = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(path)):
    k = r["Kernel_Name"].split("(")[0]
    if k.startswith("__"):
        continue
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = sorted({c for v in acc.values() for c in v})
calls = {k: max(len(x) for x in v.values()) for k, v in acc.items()}
hits = [k for k in acc if anchor in k]
base = calls[hits[0]] if hits else min(calls.values())
print(f"# per dispatch (mean); anchor {hits[0] if hits else 'fewest dispatches'}: {base} dispatches")
print("kernel".ljust(24) + "calls".rjust(7) + "".join(c.replace("SQ_", "")[:14].rjust(15) for c in cols))
for k, v in acc.items():
    print(k.replace("orbx::", "")[:24].ljust(24) + f"{calls[k]:7d}" +
          "".join((f"{sum(v[c]) / len(v[c]):15.4g}" if v[c] else " " * 15) for c in cols))
unit = "frame" if frames else "step"
print(f"# per {unit} (sum over the kernel's dispatches / anchor dispatches{' / frames' if frames else ''})")
tot = defaultdict(float)
for k, v in acc.items():
    row = {c: sum(v[c]) / base / (frames or 1.0) for c in cols if v[c]}
    for c, x in row.items():
        tot[c] += x
    print(k.replace("orbx::", "")[:24].ljust(24) + f"{calls[k] / base:7.2f}" +
          "".join((f"{row[c]:15.4g}" if c in row else " " * 15) for c in cols))
print("TOTAL".ljust(24) + " " * 7 + "".join(f"{tot[c]:15.4g}" for c in cols))
