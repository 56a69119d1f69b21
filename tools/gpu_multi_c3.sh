#!/bin/bash
# c3: serialised 1080p traces and bench lines for several library builds.
# usage: tools/gpu_multi_c3.sh <tag> <lib.so>...
set -e -o pipefail
out=gpurun_out/$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename "$lib" .so)
  ORBX_LIBRARY=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/s_$n" -o run -- python3 tools/extract_serial.py --hd > "$out/s_$n.log" 2>&1
done
for i in 1 2; do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    ORBX_LIBRARY=$PWD/$lib timeout -k 10 200 python3 bench.py --workload c3 --no-cpu-baseline --no-isolated >> "$out/b_$n.json" 2>&1
  done
done
echo multi-done
