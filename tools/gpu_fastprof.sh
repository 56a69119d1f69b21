set -e -o pipefail
mkdir -p gpurun_out/it2
export TMPDIR=/tmp
ORBX_LIBRARY=orb_slam_amd/liborbx_fastprof.so timeout -k 10 120 python3 tools/fast_phases.py > gpurun_out/it2/phases.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/it2/sq -o run -- python3 tools/extract_serial.py > gpurun_out/it2/sq.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM --output-format csv -d gpurun_out/it2/sq2 -o run -- python3 tools/extract_serial.py > gpurun_out/it2/sq2.log 2>&1
echo ok
