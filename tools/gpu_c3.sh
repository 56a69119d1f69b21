#!/bin/bash
# c3 iteration: extraction parity tests, the c3 bench line and its kernel trace.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "extract" --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
timeout -k 10 300 python3 bench.py --workload c3 --no-cpu-baseline > "$out/bench_c3.json" 2> "$out/bench_c3.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    python3 bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline --no-isolated > "$out/c3_rocprof.json" 2>&1
echo c3-done
