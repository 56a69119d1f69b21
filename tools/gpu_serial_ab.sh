#!/bin/bash
# Serialised kernel traces of liborbx.so and orb_slam_amd/liborbx_base.so (diagnostic variants).
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/snew" -o run -- python3 tools/extract_serial.py > "$out/snew.log" 2>&1
ORBX_LIBRARY=$PWD/orb_slam_amd/liborbx_base.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/sbase" -o run -- python3 tools/extract_serial.py > "$out/sbase.log" 2>&1
echo ok
