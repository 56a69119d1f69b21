"""File one tools/collect_round.sh pass (gpurun_out/round) into profiles/
under a round tag: bench lines, kernel stats, bench-under-rocprof lines,
PMC summaries (tools/pmc_summary.py, run here on the same liborbx.so that
was shipped) and SQ tables (tools/pmc_table.py).
usage: python tools/save_round.py r02"""
import glob
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
tag = sys.argv[1]
src = ROOT / "gpurun_out" / "round"
dst = ROOT / "profiles"


def one(pattern):
    hits = glob.glob(str(src / pattern), recursive=True)
    assert len(hits) == 1, (pattern, hits)
    return hits[0]


for wl in ("c2", "c3", "c5", "pose"):
    lines = [l for l in open(src / f"bench_{wl}.json") if l.startswith("{")]
    assert len(lines) == 1, wl
    (dst / f"{tag}_bench_{wl}.json").write_text(lines[0])
    shutil.copy(one(f"{wl}/trace/**/*kernel_stats.csv"), dst / f"{tag}_{wl}_kernel_stats.csv")
    shutil.copy(src / wl / "bench_under_rocprof.json", dst / f"{tag}_{wl}_bench_under_rocprof.json")
    fetch = one(f"{wl}/fetch/**/*counter_collection.csv")
    write = one(f"{wl}/write/**/*counter_collection.csv")
    sq = one(f"{wl}/sq/**/*counter_collection.csv")
    with open(dst / f"{tag}_{wl}_pmc_hbm.json", "w") as f:
        subprocess.run([sys.executable, str(ROOT / "tools/pmc_summary.py"), fetch, write, sq], stdout=f, check=True)
    with open(dst / f"{tag}_{wl}_pmc_sq.txt", "w") as f:
        subprocess.run([sys.executable, str(ROOT / "tools/pmc_table.py"), sq], stdout=f, check=True)
shutil.copy(one("c2_serial/**/*kernel_stats.csv"), dst / f"{tag}_c2_serial_kernel_stats.csv")
for wl in ("c2", "c3"):   # `bench.py --serial` profiles (tools/collect_round.sh serial), when collected
    if not (src / f"{wl}_serial_prof").exists():
        continue
    shutil.copy(one(f"{wl}_serial_prof/trace/**/*kernel_stats.csv"), dst / f"{tag}_{wl}_serial_bench_kernel_stats.csv")
    fetch = one(f"{wl}_serial_prof/fetch/**/*counter_collection.csv")
    write = one(f"{wl}_serial_prof/write/**/*counter_collection.csv")
    sq = one(f"{wl}_serial_prof/sq/**/*counter_collection.csv")
    with open(dst / f"{tag}_{wl}_serial_pmc_hbm.json", "w") as f:
        subprocess.run([sys.executable, str(ROOT / "tools/pmc_summary.py"), fetch, write, sq], stdout=f, check=True)
    with open(dst / f"{tag}_{wl}_serial_pmc_sq.txt", "w") as f:   # per dispatch and per frame
        frames = "1024" if wl == "c2" else "128"
        subprocess.run([sys.executable, str(ROOT / "tools/pmc_table.py"), sq, "--frames", frames], stdout=f,
                       check=True)
print("saved", tag)
