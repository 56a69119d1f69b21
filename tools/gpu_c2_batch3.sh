#!/bin/bash
# c2 throughput vs frames per step with the three-part pipeline (same box).
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
for b in 1024 1536 2048 1024 1536 2048; do
  timeout -k 10 200 python3 bench.py --batch $b --no-cpu-baseline --no-isolated >> "$out/b$b.json" 2>&1
done
echo ok
