#!/bin/bash
set -e -o pipefail
export TMPDIR=/tmp
for n in liborbx_base liborbx; do
  ORBX_LIBRARY=$PWD/orb_slam_amd/$n.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bfp/$n -o run -- python3 bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline --no-isolated ${BF_ARGS:-} > gpurun_out/bfp/$n.log 2>&1
done
echo done
