set -e -o pipefail
mkdir -p gpurun_out/r2a
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/gpu_tests.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2a/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/r2a/bench_c2.json 2> gpurun_out/r2a/bench_c2.err
echo done
