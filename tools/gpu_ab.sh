#!/bin/bash
# A/B of liborbx.so against orb_slam_amd/liborbx_base.so on one box:
# alternating c2 bench lines and a serialised kernel trace of each.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-isolated >> "$out/new.json" 2>&1
  ORBX_LIBRARY=$PWD/orb_slam_amd/liborbx_base.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-isolated >> "$out/base.json" 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/snew" -o run -- python3 tools/extract_serial.py > "$out/snew.log" 2>&1
ORBX_LIBRARY=$PWD/orb_slam_amd/liborbx_base.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/sbase" -o run -- python3 tools/extract_serial.py > "$out/sbase.log" 2>&1
echo ab-done
