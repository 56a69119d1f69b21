#!/bin/bash
# SQ counters of the c3 bench (1920x1080) for the FAST kernel.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d "$out/lds" -o run -- python3 bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-isolated > "$out/lds.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM --output-format csv -d "$out/act" -o run -- python3 bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-isolated > "$out/act.log" 2>&1
echo pmc-done
