"""Summarise a tools/gpu_ab.sh run: bench values and per-kernel averages."""
import csv, glob, json, sys

d = sys.argv[1]
for v in ("new", "base"):
    vals = [json.loads(l)["value"] for l in open(f"{d}/{v}.json") if l.startswith("{")]
    print(v, " ".join(f"{x:.0f}" for x in vals))
for v in ("snew", "sbase"):
    f = glob.glob(f"{d}/{v}/**/*kernel_stats.csv", recursive=True)[0]
    print(v, "  ".join(f"{r['Name'].split('(')[0].replace('void orbx::', '')[:22]}={float(r['TotalDurationNs'])/float(r['Calls'])/1e3:.1f}"
                      for r in csv.DictReader(open(f))))
