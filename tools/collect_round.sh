#!/bin/bash
# One GPU-box pass over everything the round reports (run from the repo
# root): the GPU test suite, smoke(), the default bench line, the pose
# bench, and the rocprofv3 summaries behind them (c2: kernel trace + stats,
# FETCH_SIZE and WRITE_SIZE in separate passes; pose: kernel trace + stats).
# Every GPU step has its own time limit; the first failure ends the script.
set -e -o pipefail
out=gpurun_out/round
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 300 python3 bench.py > "$out/bench_c2.json" 2> "$out/bench_c2.err"
timeout -k 10 300 python3 bench.py --workload pose --cpu-budget 10 > "$out/bench_pose.json" 2> "$out/bench_pose.err"
tools/collect_profiles.sh "$out/c2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/pose_trace" -o run -- \
    python3 bench.py --workload pose --steps 10 --warmup 2 --no-cpu-baseline > "$out/pose_under_rocprof.json"
echo round-collected
