#!/bin/bash
# Extraction parity tests, then c3 and c2 A/B (liborbx.so vs liborbx_base.so).
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -k "extract or fast or bench_shape or sort_era or contract" --timeout 200 --timeout-method thread > "$out/tests.log" 2>&1
tools/gpu_ab.sh "$1/c3" c3 --hd
tools/gpu_ab.sh "$1/c2" c2
echo band-done
