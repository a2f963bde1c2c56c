set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo smoke_ok >> gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench1.json > gpurun_out/bench1.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof1.log 2>&1
echo done
