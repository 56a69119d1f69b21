#!/bin/bash
# Parity tests selected by -k, then tools/gpu_ab.sh (liborbx.so vs liborbx_base.so).
# usage: tools/gpu_test_ab.sh <tag> <pytest -k expr> [workload] [extract_serial.py args]
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -k "$2" --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
tools/gpu_ab.sh "$1" "${3:-c2}" "${4:-}"
