#!/bin/bash
# c2 throughput by batch size with the staged (mode 0) and fused (mode 1) pyramid.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
for m in 0 1; do for b in 256 512 1024; do
timeout -k 10 200 python3 bench.py --pyramid-mode $m --batch $b --no-cpu-baseline --no-isolated > "$out/m${m}_b$b.json" 2>&1
done; done
echo ok
