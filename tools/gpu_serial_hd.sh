#!/bin/bash
# Serialised kernel trace of the 1080p (c3) extraction + brute-force match.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/shd" -o run -- python3 tools/extract_serial.py --hd > "$out/shd.log" 2>&1
echo ok
