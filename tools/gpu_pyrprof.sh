#!/bin/bash
# Fused pyramid phase breakdown (ORBX_PYR_PROFILE build) at 640x480.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
ORBX_PYR_VERBOSE=1 ORBX_LIBRARY=orb_slam_amd/liborbx_pyrprof.so timeout -k 10 120 python3 tools/pyr_phases.py > "$out/phases.txt" 2>&1
echo ok
