#!/bin/bash
# Serialised kernel traces (tools/extract_serial.py) only, for several builds.
# usage: tools/gpu_serial_libs.sh <tag> <lib.so>...   (EXTRA: --hd for 1080p)
set -e -o pipefail
out=gpurun_out/$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename "$lib" .so)
  ORBX_LIBRARY=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/s_$n" -o run -- python3 tools/extract_serial.py ${EXTRA:-} > "$out/s_$n.log" 2>&1
done
echo serial-libs-done
