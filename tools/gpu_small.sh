#!/bin/bash
# c2 vs ORBX_SMALL_PX (small top pyramid levels in one per-frame launch), same box.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
ORBX_SMALL_PX=80000 timeout -k 10 300 python3 -u -m pytest tests/test_extract_gpu.py -m gpu -x -q -k "matches_oracle or configs or ragged" --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
for px in 0 40000 80000 0 40000 80000; do
  ORBX_SMALL_PX=$px timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-isolated >> "$out/p$px.json" 2>&1
done
for px in 0 80000; do
  ORBX_SMALL_PX=$px timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/s$px" -o run -- python3 tools/extract_serial.py > "$out/s$px.log" 2>&1
done
echo ok
