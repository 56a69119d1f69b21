#!/bin/bash
# round 4: extraction parity tests, then c2 x2 and c3 bench lines (no CPU legs)
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_extract_gpu.py \
    tests/test_golden.py tests/test_bench_shape_gpu.py > "$out/tests.log" 2>&1
for r in 1 2; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline --verbose > "$out/c2_$r.json" 2> "$out/c2_$r.err"
done
timeout -k 10 200 python3 bench.py --workload c3 --no-cpu-baseline --verbose > "$out/c3.json" 2> "$out/c3.err"
echo done
