#!/bin/bash
# A/B of liborbx.so against orb_slam_amd/liborbx_base.so on one box:
# alternating bench lines and a serialised kernel trace of each.
# usage: tools/gpu_ab.sh <tag> [workload (c2)] [extract_serial.py args]
set -e -o pipefail
out=gpurun_out/$1
wl=${2:-c2}
sargs=${3:-}
mkdir -p "$out"
export TMPDIR=/tmp
base=$PWD/orb_slam_amd/liborbx_base.so
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --workload "$wl" --no-cpu-baseline --no-isolated >> "$out/new.json" 2>&1
  ORBX_LIBRARY=$base timeout -k 10 200 python3 bench.py --workload "$wl" --no-cpu-baseline --no-isolated >> "$out/base.json" 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/snew" -o run -- python3 tools/extract_serial.py $sargs > "$out/snew.log" 2>&1
ORBX_LIBRARY=$base timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/sbase" -o run -- python3 tools/extract_serial.py $sargs > "$out/sbase.log" 2>&1
echo ab-done
