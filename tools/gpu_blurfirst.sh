#!/bin/bash
# c2 with each pipeline part's blur before its FAST (ORBX_BLUR_FIRST) vs after retain, same box.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
ORBX_BLUR_FIRST=1 timeout -k 10 300 python3 -u -m pytest tests/test_extract_gpu.py -m gpu -x -q -k "large_batch or pipeline" --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-isolated >> "$out/after.json" 2>&1
  ORBX_BLUR_FIRST=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-isolated >> "$out/first.json" 2>&1
  ORBX_LIBRARY=$PWD/orb_slam_amd/liborbx_base.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-isolated >> "$out/base.json" 2>&1
done
echo ok
