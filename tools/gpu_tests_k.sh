#!/bin/bash
# GPU tests selected by -k.  usage: tools/gpu_tests_k.sh <tag> <pytest -k expr>
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v -k "$2" --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
echo tests-done
