#!/bin/bash
# Local BA diagnostics: host-side phase times of the c5 bench (stderr) and
# the kernel's phase breakdown (ORBX_LBA_PROFILE build, tools/lba_phases.py).
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
ORBX_LBA_PROFILE_HOST=1 timeout -k 10 200 python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-isolated > "$out/c5.json" 2> "$out/c5_host.txt"
if [ -f orb_slam_amd/liborbx_lbaprof.so ]; then
ORBX_LIBRARY=orb_slam_amd/liborbx_lbaprof.so timeout -k 10 200 python3 tools/lba_phases.py > "$out/lba_phases.txt" 2>&1
fi
echo ok
