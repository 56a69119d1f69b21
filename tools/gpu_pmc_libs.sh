#!/bin/bash
# LDS / issue counters of the serialised extraction for several library builds
# (diagnostic variants).  usage: tools/gpu_pmc_libs.sh <tag> <lib.so>...
set -e -o pipefail
out=gpurun_out/$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename "$lib" .so)
  ORBX_LIBRARY=$PWD/$lib timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d "$out/p_$n" -o run -- python3 tools/extract_serial.py > "$out/p_$n.log" 2>&1
  ORBX_LIBRARY=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/s_$n" -o run -- python3 tools/extract_serial.py > "$out/s_$n.log" 2>&1
done
echo pmc-libs-done
