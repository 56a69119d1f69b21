#!/bin/bash
# Fused-pyramid iteration on the GPU box: extraction parity tests, the phase
# profile (ORBX_PYR_PROFILE build), the default bench line and a serialised
# kernel trace.  usage: tools/gpu_pyr_iter.sh <tag>
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k extract --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
ORBX_PYR_VERBOSE=1 ORBX_LIBRARY=orb_slam_amd/liborbx_pyrprof.so timeout -k 10 120 python3 tools/pyr_phases.py > "$out/phases.txt" 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$out/bench.json" 2> "$out/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/serial" -o run -- \
    python3 tools/extract_serial.py > "$out/serial.log" 2>&1
echo iter-done
