#!/bin/bash
# One GPU-box pass over what the round reports (run from the repo root).
#   part 1: the GPU test suite, smoke(), the four bench lines (c2 default,
#           pose, c3, c5, each with a bounded cpu_baseline), a --gpus 2 c2
#           line (both ranks on the box's one GPU), and the
#           serialised c2 kernel trace (tools/extract_serial.py)
#   part 2: tools/collect_profiles.sh for c2, c3, c5, pose (kernel trace +
#           stats, FETCH_SIZE, WRITE_SIZE and one SQ pass each)
#   serial: the same for `bench.py --serial` at c2 and c3 (one launch per
#           kernel over the whole batch: the bench line's headline roofline)
# usage: tools/collect_round.sh 1|2|serial|bench ; every GPU step has its own time limit
# and the first failure ends the script.
set -e -o pipefail
out=gpurun_out/round
mkdir -p "$out"
export TMPDIR=/tmp
if [ "$1" = bench ]; then   # the four bench lines only (after the profiles exist)
timeout -k 10 300 python3 bench.py > "$out/bench_c2.json" 2> "$out/bench_c2.err"
timeout -k 10 300 python3 bench.py --workload pose --cpu-budget 10 > "$out/bench_pose.json" 2> "$out/bench_pose.err"
timeout -k 10 300 python3 bench.py --workload c3 --cpu-budget 10 > "$out/bench_c3.json" 2> "$out/bench_c3.err"
timeout -k 10 300 python3 bench.py --workload c5 --cpu-budget 10 > "$out/bench_c5.json" 2> "$out/bench_c5.err"
elif [ "$1" = 1 ]; then
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 300 python3 bench.py > "$out/bench_c2.json" 2> "$out/bench_c2.err"
timeout -k 10 300 python3 bench.py --workload pose --cpu-budget 10 > "$out/bench_pose.json" 2> "$out/bench_pose.err"
timeout -k 10 300 python3 bench.py --workload c3 --cpu-budget 10 > "$out/bench_c3.json" 2> "$out/bench_c3.err"
timeout -k 10 300 python3 bench.py --workload c5 --cpu-budget 10 > "$out/bench_c5.json" 2> "$out/bench_c5.err"
timeout -k 10 300 python3 bench.py --gpus 2 --cpu-budget 4 > "$out/bench_c2_gpus2.json" 2> "$out/bench_c2_gpus2.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/c2_serial" -o run -- \
    python3 tools/extract_serial.py > "$out/c2_serial.log" 2>&1
elif [ "$1" = serial ]; then   # PMC of the serialised bench (the headline roofline's launch)
tools/collect_profiles.sh "$out/c2_serial_prof" --serial
tools/collect_profiles.sh "$out/c3_serial_prof" --workload c3 --serial
else
tools/collect_profiles.sh "$out/c2"
tools/collect_profiles.sh "$out/c3" --workload c3
tools/collect_profiles.sh "$out/pose" --workload pose
tools/collect_profiles.sh "$out/c5" --workload c5
fi
echo round-collected
