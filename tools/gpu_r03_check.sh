#!/bin/bash
# Round-3 GPU pass: the whole -m gpu suite, then the default bench line.
set -e -o pipefail
out=gpurun_out/r03_check
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/gpu_tests.log" 2>&1
timeout -k 10 300 python3 bench.py > "$out/bench_c2.json" 2> "$out/bench_c2.err"
echo done
