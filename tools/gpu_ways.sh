#!/bin/bash
# c2 throughput with the extraction pipeline in 2, 3 and 4 parts (bench.py --split-ways).
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "pipeline or large_batch or operator_call" --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
for w in 2 3 4; do
timeout -k 10 200 python3 bench.py --split-ways $w --no-cpu-baseline --no-isolated > "$out/w$w.json" 2>&1
timeout -k 10 200 python3 bench.py --split-ways $w --workload c3 --no-cpu-baseline --no-isolated > "$out/c3_w$w.json" 2>&1
done
echo ok
