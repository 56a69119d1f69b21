#!/bin/bash
# FAST iteration: extraction parity tests, then A/B vs liborbx_base.so
# (bench lines + serialised traces), SQ counters of both serialised runs and
# both phase breakdowns.  usage: tools/gpu_fast_iter.sh <tag>
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -k "extract or nth or fast" --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
tools/gpu_ab.sh "$1"
tools/gpu_fast_diag.sh "$1"
