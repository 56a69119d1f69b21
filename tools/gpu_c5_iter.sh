#!/bin/bash
# Local BA iteration: parity tests, the c5 bench line (and an optional
# variant library), one FETCH_SIZE pass over a short c5 run.
set -e -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "lba" --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
timeout -k 10 200 python3 bench.py --workload c5 --no-cpu-baseline --no-isolated > "$out/c5.json" 2>&1
if [ -n "$2" ]; then
ORBX_LIBRARY=$2 timeout -k 10 200 python3 bench.py --workload c5 --no-cpu-baseline --no-isolated > "$out/c5_variant.json" 2>&1
fi
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
    python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline --no-isolated --no-kernel-timing > "$out/fetch.log" 2>&1
echo ok
