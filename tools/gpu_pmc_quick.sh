#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ instruction mix) of one bench
# command, each in its own rocprofv3 run.  usage: tools/gpu_pmc_quick.sh <out> [bench args]
set -e -o pipefail
out=gpurun_out/$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated "$@" > "$out/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated "$@" > "$out/write.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$out/sq" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated "$@" > "$out/sq.log" 2>&1
echo ok
