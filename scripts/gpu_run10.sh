set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_components.py tests/test_gpu_golden.py -m gpu -x -q -p no:cacheprovider -k "conv" > gpurun_out/pytest10.log 2>&1 || { echo "pytest_rc=$?" >> gpurun_out/pytest10.log; exit 3; }
timeout -k 10 100 python scripts/microbench.py --reps 20 --only bwd_fused > gpurun_out/micro10.log 2>&1 || exit 5

echo done
