"""Summarise bench JSON lines of one GPU A/B directory: value, ms per step and
the serialised per-kernel times (python3 tools/bench_lines.py gpurun_out/<dir>)."""
import json
import sys
from pathlib import Path

for f in sorted(Path(sys.argv[1]).glob("*.json")):
    lines = f.read_text().strip().splitlines()
    if not lines:
        continue
    d = json.loads(lines[-1])
    ser = (d.get("kernels") or {}).get("serial") or {}
    ks = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in ser.items() if isinstance(v, dict) and v.get("launches"))
    print(f"{f.name:28s} {d['value']:>12} {d['ms_per_step']:>8}  {ks}")
