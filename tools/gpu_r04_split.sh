#!/bin/bash
# round 4: c2 bench lines at 2 / 3 / 4 extraction pipeline parts, twice each
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
for r in 1 2; do
for w in 2 3 4; do
timeout -k 10 200 python3 bench.py --split-ways $w --no-cpu-baseline > "$out/c2_w${w}_$r.json" 2> "$out/c2_w${w}_$r.err"
done
done
echo done
