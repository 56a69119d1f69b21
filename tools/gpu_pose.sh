#!/bin/bash
# Pose iteration: pose parity tests, the pose bench line, its kernel trace.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "pose" --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
timeout -k 10 300 python3 bench.py --workload pose --no-cpu-baseline > "$out/bench_pose.json" 2> "$out/bench_pose.err"
echo pose-done
