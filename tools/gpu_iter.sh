#!/bin/bash
# Iteration pass on the GPU box (repo root): extraction parity tests, the
# default bench line, and a serialised kernel trace of tools/extract_serial.py.
# usage: tools/gpu_iter.sh <tag> [pytest -k expr]
set -e -o pipefail
tag=$1; k=${2:-extract}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "$k" --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$out/bench.json" 2> "$out/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/serial" -o run -- \
    python3 tools/extract_serial.py > "$out/serial.log" 2>&1
echo iter-done
