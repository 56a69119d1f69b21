#!/bin/bash
# round 4: local-BA phase stamps (iteration and k_lba_build) of the profile build
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
ORBX_LIBRARY=orb_slam_amd/liborbx_lbaprof.so timeout -k 10 200 python3 tools/lba_phases.py 256 > "$out/phases_256.txt" 2>&1
echo done
