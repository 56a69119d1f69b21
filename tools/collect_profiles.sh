#!/bin/bash
# Collect the rocprofv3 summaries behind bench.py's numbers (run on the GPU
# box from the repo root): kernel trace + stats of the bench command, then
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md:
# the two TCC counters do not fit one pass; no trace domains with --pmc), and
# one SQ instruction / wave-state pass.
# usage: tools/collect_profiles.sh <out dir under gpurun_out> [bench args...]
set -e -o pipefail
out=$1; shift
export TMPDIR=/tmp
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-isolated --verbose "$@" > "$out/bench_under_rocprof.json"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated "$@" > "$out/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated "$@" > "$out/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$out/sq" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated "$@" > "$out/sq.log" 2>&1
echo collected
