"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (TCC_EA0_RDREQ/WRREQ based).
gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half
the bytes of a wide coalesced streaming read (16 B per lane); other access
widths are uncalibrated.  Both figures are kept: hbm_bytes_raw (FETCH + WRITE
as counted) and hbm_bytes_fetch_x2 (the streaming-read correction).  For a
kernel whose reads are not wide coalesced streams (gathers, scattered 8-B
rows, atomics) the truth lies between the two.
The summary records the build it profiled (`_meta`: git HEAD and the SHA-256
of orb_slam_amd/liborbx.so as shipped to the GPU box), so bench.py can refuse
a stale profile.
usage: python tools/pmc_summary.py <fetch run_counter_collection.csv> <write csv> [<SQ csv>]
(the optional third pass adds SQ_INSTS_VALU per dispatch -- bench.py's
roofline_valu -- and its sum over all of the kernel's dispatches per step,
a step being one k_fast_cells dispatch: the resize runs once per level)
"""
import csv
import hashlib
import json
import subprocess
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def build_id():
    lib = ROOT / "orb_slam_amd" / "liborbx.so"
    sha = hashlib.sha256(lib.read_bytes()).hexdigest() if lib.exists() else None
    try:
        head = subprocess.run(["git", "-C", str(ROOT), "rev-parse", "--short=12", "HEAD"], capture_output=True,
                              text=True).stdout.strip() or None
    except OSError:
        head = None
    return {"git_head": head, "liborbx_sha256": sha}


def load_all(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return acc


def load(path, counter):
    return {k: sum(v) / len(v) for k, v in load_all(path, counter).items()}


def per_step(acc, anchor="k_fast_cells"):
    """Sum over each kernel's dispatches per anchor dispatch (one per step):
    a kernel launched several times a step (the resize, once per level)
    counts all of its launches."""
    hits = [k for k in acc if anchor in k]
    base = len(acc[hits[0]]) if hits else min(len(v) for v in acc.values())
    return {k: (sum(v) / base, len(v) / base) for k, v in acc.items()}


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    valu_all = load_all(sys.argv[3], "SQ_INSTS_VALU") if len(sys.argv) > 3 else {}
    valu = {k: sum(v) / len(v) for k, v in valu_all.items()}
    valu_step = per_step({k: v for k, v in valu_all.items() if not k.startswith("__amd")}) if valu_all else {}
    out = {"_meta": build_id()}
    for k in sorted(set(fetch) | set(write)):
        if k.startswith("__amd"):
            continue
        fk, wk = fetch.get(k, 0.0), write.get(k, 0.0)
        out[k] = {"FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk,
                  "hbm_bytes_raw": (fk + wk) * 1024, "hbm_bytes_fetch_x2": (2 * fk + wk) * 1024}
        if k in valu:
            out[k]["SQ_INSTS_VALU"] = valu[k]   # mean per dispatch
            out[k]["SQ_INSTS_VALU_per_step"], out[k]["dispatches_per_step"] = valu_step[k]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
