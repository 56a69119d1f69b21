#!/bin/bash
# Matching iteration: match / search parity tests, the default c2 bench line,
# the serialised kernel trace.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "match or search or init or smoke or extract" --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$out/bench.json" 2> "$out/bench.err"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-isolated --sync-match > "$out/bench_sync.json" 2> "$out/bench_sync.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/serial" -o run -- \
    python3 tools/extract_serial.py > "$out/serial.log" 2>&1
echo ok
