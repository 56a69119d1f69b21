#!/bin/bash
# c3 throughput by batch size.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
for b in 64 128 256; do
timeout -k 10 200 python3 bench.py --workload c3 --batch $b --no-cpu-baseline --no-isolated > "$out/b$b.json" 2>&1
done
echo ok
