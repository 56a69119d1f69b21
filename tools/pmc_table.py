"""Per-kernel mean of every counter in a rocprofv3 --pmc CSV (one table).
usage: python tools/pmc_table.py <run_counter_collection.csv>"""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = sorted({c for v in acc.values() for c in v})
print("kernel".ljust(24) + "".join(c.replace("SQ_", "")[:14].rjust(15) for c in cols))
for k, v in acc.items():
    if k.startswith("__"):
        continue
    print(k.replace("orbx::", "")[:24].ljust(24) +
          "".join((f"{sum(v[c]) / len(v[c]):15.4g}" if v[c] else " " * 15) for c in cols))
