#!/bin/bash
# Kernel trace (per-dispatch timestamps) of a short c2 bench run.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out/tl" -o run -- \
    python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-isolated --no-kernel-timing > "$out/bench.json" 2>&1
echo tl-done
