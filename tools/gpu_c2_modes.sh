#!/bin/bash
# c2 pipeline diagnostics: async vs sync matching, and a per-dispatch kernel
# trace of a short default run (tools/timeline_summary.py reads it).
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-isolated > "$out/async.json" 2>&1
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-isolated --sync-match > "$out/sync.json" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out/tl" -o run -- \
    python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-isolated --no-kernel-timing > "$out/tl_bench.json" 2>&1
echo ok
