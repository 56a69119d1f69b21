#!/bin/bash
# Local BA check on one box: the GPU tests, the c5 bench line (default build
# and, when present, the kSchurGroup = 1 build), and the kernel's phase
# breakdown (ORBX_LBA_PROFILE build, tools/lba_phases.py).
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_lba_gpu.py -x -q --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
timeout -k 10 200 python3 bench.py --workload c5 --no-cpu-baseline --steps 10 > "$out/c5.json" 2> "$out/c5.err"
if [ -f orb_slam_amd/liborbx_g1.so ]; then
ORBX_LIBRARY=orb_slam_amd/liborbx_g1.so timeout -k 10 200 python3 bench.py --workload c5 --no-cpu-baseline --steps 10 > "$out/c5_g1.json" 2> "$out/c5_g1.err"
fi
ORBX_LIBRARY=orb_slam_amd/liborbx_lbaprof.so timeout -k 10 200 python3 tools/lba_phases.py > "$out/lba_phases.txt" 2>&1
echo ok
