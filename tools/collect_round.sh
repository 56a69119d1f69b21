#!/bin/bash
# One GPU-box pass over everything the round reports (run from the repo
# root): the GPU test suite, smoke(), the default bench line, the c3, c5 and
# pose bench lines, and the rocprofv3 summaries behind them (c2: kernel trace
# + stats, FETCH_SIZE and WRITE_SIZE in separate passes, one SQ instruction
# pass; c5 and pose: kernel trace + stats).
# Every GPU step has its own time limit; the first failure ends the script.
set -e -o pipefail
out=gpurun_out/round
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 300 python3 bench.py > "$out/bench_c2.json" 2> "$out/bench_c2.err"
timeout -k 10 300 python3 bench.py --workload pose --cpu-budget 10 > "$out/bench_pose.json" 2> "$out/bench_pose.err"
timeout -k 10 300 python3 bench.py --workload c3 --cpu-budget 10 > "$out/bench_c3.json" 2> "$out/bench_c3.err"
timeout -k 10 300 python3 bench.py --workload c5 --cpu-budget 10 > "$out/bench_c5.json" 2> "$out/bench_c5.err"
tools/collect_profiles.sh "$out/c2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$out/c2_sq" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated > "$out/c2_sq.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/c5_trace" -o run -- \
    python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > "$out/c5_under_rocprof.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/pose_trace" -o run -- \
    python3 bench.py --workload pose --steps 10 --warmup 2 --no-cpu-baseline > "$out/pose_under_rocprof.json"
echo round-collected
