#!/bin/bash
set -e -o pipefail
out=gpurun_out/tsweep
mkdir -p "$out"
export TMPDIR=/tmp
for T in 4 8 16 24; do
ORBX_PYR_T=$T ORBX_PYR_VERBOSE=1 ORBX_LIBRARY=orb_slam_amd/liborbx_pyrprof.so timeout -k 10 120 python3 tools/pyr_phases.py > "$out/phases_T$T.txt" 2>&1
done
echo ok
