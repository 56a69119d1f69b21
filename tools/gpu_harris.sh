#!/bin/bash
# Harris-score parity + the default extraction tests.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_extract_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
echo ok
