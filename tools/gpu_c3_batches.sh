#!/bin/bash
# c3 bench lines at several batch sizes (pairs per step).  usage: tools/gpu_c3_batches.sh <tag> <batch>...
set -e -o pipefail
out=gpurun_out/$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
for i in 1 2; do
  for b in "$@"; do
    timeout -k 10 200 python3 bench.py --workload c3 --batch "$b" --no-cpu-baseline --no-isolated >> "$out/b_$b.json" 2>&1
  done
done
echo c3b-done
