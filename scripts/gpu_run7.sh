set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --json-out gpurun_out/bench7.json > gpurun_out/bench7.log 2>&1 || exit 3
timeout -k 10 300 python scripts/microbench.py --reps 20 > gpurun_out/micro7.log 2>&1 || exit 4
echo done
