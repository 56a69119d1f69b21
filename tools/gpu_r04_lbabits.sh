#!/bin/bash
# round 4: local-BA solves of two builds written for a bit-for-bit comparison
# (tools/lba_bits.py), then the A/B of tools/gpu_r04_lbaab.sh
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/lba_bits.py "$out/bits_main.npz" > "$out/bits_main.log" 2>&1
ORBX_LIBRARY=orb_slam_amd/$2 timeout -k 10 200 python3 tools/lba_bits.py "$out/bits_var.npz" > "$out/bits_var.log" 2>&1
bash tools/gpu_r04_lbaab.sh "$1" "$2"
