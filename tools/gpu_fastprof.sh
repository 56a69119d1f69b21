#!/bin/bash
# FAST phase breakdown (ORBX_FAST_PROFILE build) at 640x480 and 1920x1080.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
ORBX_LIBRARY=orb_slam_amd/liborbx_fastprof.so timeout -k 10 120 python3 tools/fast_phases.py > "$out/phases_c2.txt" 2>&1
ORBX_LIBRARY=orb_slam_amd/liborbx_fastprof.so timeout -k 10 120 python3 tools/fast_phases.py 1920 1080 2000 32 > "$out/phases_c3.txt" 2>&1
echo ok
