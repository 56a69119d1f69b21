#!/bin/bash
# round 4: chunked FAST (next tile prefetched by global_load_lds) -- parity
# tests, then c2 bench lines at chunk 1 / 2 / 4 / 8 on the same box
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_extract_gpu.py \
    tests/test_golden.py > "$out/tests.log" 2>&1
for c in 1 2 4 8 1 4; do
timeout -k 10 200 python3 bench.py --fast-chunk $c --no-cpu-baseline --verbose > "$out/c2_k$c.json" 2> "$out/c2_k$c.err"
cp "$out/c2_k$c.json" "$out/c2_k${c}_$(date +%s%N).json"
done
echo done
