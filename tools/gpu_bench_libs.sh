#!/bin/bash
# Bench lines (c2 unless BENCH_ARGS says otherwise) for several library builds,
# interleaved twice.  usage: tools/gpu_bench_libs.sh <tag> <lib.so>...
set -e -o pipefail
out=gpurun_out/$1; shift
mkdir -p "$out"
for i in 1 2; do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    ORBX_LIBRARY=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-isolated ${BENCH_ARGS:-} >> "$out/b_$n.json" 2>/dev/null
  done
done
echo bench-libs-done
