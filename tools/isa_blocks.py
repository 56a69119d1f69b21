"""Static instruction counts per basic block of one kernel in a gfx950 .s file.

Usage: python tools/isa_blocks.py <file.s> <kernel-symbol-substring>
Emit the assembly with hipcc --cuda-device-only -S (same flags as build.py).
Prints VALU / SALU / LDS / global counts per block and marks back edges (loops).
"""
import re
import sys


def main(path, name):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(name) + r"\S*:", l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, blk = [], None
    for i in range(start, end):
        s = lines[i].strip()
        m = re.match(r"^(\.LBB\d+_\d+):", s)
        if m or blk is None:
            blk = {"name": m.group(1) if m else "entry", "line": i + 1, "v": 0, "s": 0, "ds": 0, "gl": 0, "br": []}
            blocks.append(blk)
            if m:
                continue
        if not s or s[0] in ";.":
            continue
        op = s.split()[0]
        if op.startswith("v_"):
            blk["v"] += 1
        elif op.startswith("ds_"):
            blk["ds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            blk["gl"] += 1
        elif op.startswith("s_") and "branch" not in op and not op.startswith(("s_waitcnt", "s_nop")):
            blk["s"] += 1
        if "branch" in op:
            blk["br"].append(s.split()[-1])
    order = {b["name"]: k for k, b in enumerate(blocks)}
    for k, b in enumerate(blocks):
        back = [t for t in b["br"] if t in order and order[t] <= k]
        print(f"{b['name']:14s} L{b['line']:6d} valu={b['v']:4d} salu={b['s']:3d} ds={b['ds']:3d} gl={b['gl']:2d}"
              f" -> {','.join(b['br'])}{'  LOOP' if back else ''}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
