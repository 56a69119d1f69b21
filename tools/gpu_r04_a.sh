#!/bin/bash
# round 4, first pass: the era / golden / bench-shape GPU tests, the default
# bench line, and `bench.py --gpus 2` (two ranks on the box's one GPU, gloo)
set -e -o pipefail
out=gpurun_out/r04a
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_sort_era.py tests/test_golden.py tests/test_nth_gpu.py tests/test_bench_shape_gpu.py > "$out/tests.log" 2>&1
timeout -k 10 300 python3 bench.py > "$out/bench_c2.json" 2> "$out/bench_c2.err"
timeout -k 10 400 python3 bench.py --gpus 2 > "$out/bench_c2_gpus2.json" 2> "$out/bench_c2_gpus2.err"
echo done
