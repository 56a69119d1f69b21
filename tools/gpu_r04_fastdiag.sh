#!/bin/bash
# round 4: FAST phase stamps (ORBX_FAST_PROFILE build) and LDS / issue
# counters of the serialised extraction
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
ORBX_LIBRARY=orb_slam_amd/liborbx_fastprof.so timeout -k 10 120 python3 tools/fast_phases.py > "$out/phases_c2.txt" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$out/lds" -o run -- python3 tools/extract_serial.py > "$out/lds.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAVES --output-format csv -d "$out/act" -o run -- python3 tools/extract_serial.py > "$out/act.log" 2>&1
echo done
