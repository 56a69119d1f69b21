#!/bin/bash
# round 4: c2 bench lines at 512 / 1024 / 2048 / 4096 frames per step, twice each
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
for r in 1 2; do
for b in 512 1024 2048 4096; do
timeout -k 10 200 python3 bench.py --batch $b --no-cpu-baseline > "$out/c2_b${b}_$r.json" 2> "$out/c2_b${b}_$r.err"
done
done
echo done
