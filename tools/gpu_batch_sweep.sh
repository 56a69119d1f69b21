set -e -o pipefail
mkdir -p gpurun_out/bs
for b in 64 128 256 512; do timeout -k 10 200 python3 bench.py --batch $b --no-cpu-baseline --no-isolated > gpurun_out/bs/b$b.json 2>&1; done
echo ok
