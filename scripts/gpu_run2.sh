set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; echo "pytest_rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --json-out gpurun_out/bench2.json > gpurun_out/bench2.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof2.log 2>&1
echo done
