#!/bin/bash
# round 4: local BA v2 -- parity tests, the c5 bench line, the phase profile
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_lba_gpu.py \
    tests/test_golden.py tests/test_bench_shape_gpu.py -k "lba or c5" > "$out/tests.log" 2>&1
timeout -k 10 300 python3 bench.py --workload c5 --cpu-budget 4 --cpu-protocol 5,40 > "$out/bench_c5.json" 2> "$out/bench_c5.err"
ORBX_LIBRARY=orb_slam_amd/liborbx_lbaprof.so timeout -k 10 200 python3 tools/lba_phases.py 256 > "$out/phases_256.txt" 2>&1
echo done
