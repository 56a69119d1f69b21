#!/bin/bash
# round 4: local-BA A/B -- parity tests of the default build, then c5 lines of
# the default build and of a variant library, twice each; FAST phase stamps
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_lba_gpu.py \
    tests/test_golden.py tests/test_bench_shape_gpu.py -k "lba or c5" > "$out/tests.log" 2>&1
for r in 1 2; do
timeout -k 10 200 python3 bench.py --workload c5 --no-cpu-baseline > "$out/c5_main_$r.json" 2> "$out/c5_main_$r.err"
ORBX_LIBRARY=orb_slam_amd/$2 timeout -k 10 200 python3 bench.py --workload c5 --no-cpu-baseline > "$out/c5_var_$r.json" 2> "$out/c5_var_$r.err"
done
ORBX_LIBRARY=orb_slam_amd/liborbx_lbaprof.so timeout -k 10 200 python3 tools/lba_phases.py 256 > "$out/phases_256.txt" 2>&1
ORBX_LIBRARY=orb_slam_amd/liborbx_fastprof.so timeout -k 10 120 python3 tools/fast_phases.py > "$out/fast_phases_c2.txt" 2>&1
echo done
