#!/bin/bash
# FAST diagnosis, new build vs base: SQ counters of the serialised extraction
# (tools/extract_serial.py) and the ORBX_FAST_PROFILE phase breakdown.
# usage: tools/gpu_fast_diag.sh <tag>   (needs liborbx_base.so, liborbx_fastprof.so, liborbx_fastprof_base.so)
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
base=$PWD/orb_slam_amd/liborbx_base.so
ctrs="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU"
timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$out/sq_new" -o run -- python3 tools/extract_serial.py > "$out/sq_new.log" 2>&1
ORBX_LIBRARY=$base timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$out/sq_base" -o run -- python3 tools/extract_serial.py > "$out/sq_base.log" 2>&1
ORBX_LIBRARY=orb_slam_amd/liborbx_fastprof.so timeout -k 10 120 python3 tools/fast_phases.py > "$out/phases_new.txt" 2>&1
ORBX_LIBRARY=orb_slam_amd/liborbx_fastprof_base.so timeout -k 10 120 python3 tools/fast_phases.py > "$out/phases_base.txt" 2>&1
echo diag-done
