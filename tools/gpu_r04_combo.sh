#!/bin/bash
# round 4: local-BA parity + c5 line + phases, then the FAST phase stamps
set -e -o pipefail
tools/gpu_r04_lba.sh "$1"
out=gpurun_out/$1
ORBX_LIBRARY=orb_slam_amd/liborbx_fastprof.so timeout -k 10 120 python3 tools/fast_phases.py > "$out/fast_phases_c2.txt" 2>&1
echo combo-done
