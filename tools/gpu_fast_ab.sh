#!/bin/bash
# Extraction A/B on one box: extraction parity tests, the default c2 bench
# line, the serialised per-kernel times (bench.py --serial --verbose) and
# FAST's phase breakdown (ORBX_FAST_PROFILE build, tools/fast_phases.py).
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_extract_gpu.py tests/test_match_gpu.py -x -q --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
timeout -k 10 200 python3 bench.py --no-cpu-baseline > "$out/c2.json" 2> "$out/c2.err"
timeout -k 10 200 python3 bench.py --no-cpu-baseline --serial --verbose --steps 5 > "$out/c2_serial.json" 2> "$out/c2_serial.err"
if [ -f orb_slam_amd/liborbx_fastprof.so ]; then
ORBX_LIBRARY=orb_slam_amd/liborbx_fastprof.so timeout -k 10 200 python3 tools/fast_phases.py > "$out/fast_phases.txt" 2>&1
fi
echo ok
