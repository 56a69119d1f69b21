#!/bin/bash
# round 4: local-BA (c5) HBM traffic and LDS counters of the current build
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
    python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-isolated > "$out/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
    python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-isolated > "$out/write.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$out/lds" -o run -- \
    python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-isolated > "$out/lds.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES --output-format csv -d "$out/act" -o run -- \
    python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-isolated > "$out/act.log" 2>&1
echo done
