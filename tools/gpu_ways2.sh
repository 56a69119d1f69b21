#!/bin/bash
# c2 pipeline parts: repeat runs of the 3-part default against 2 parts, with
# the extraction / matching parity tests.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "extract or match or pipeline or smoke" --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
for rep in 1 2; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-isolated > "$out/w3_r$rep.json" 2>&1
timeout -k 10 200 python3 bench.py --split-ways 2 --no-cpu-baseline --no-isolated > "$out/w2_r$rep.json" 2>&1
done
timeout -k 10 200 python3 bench.py --batch 1536 --no-cpu-baseline --no-isolated > "$out/w3_b1536.json" 2>&1
echo ok
