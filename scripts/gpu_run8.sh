set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu8.log 2>&1 || { echo "pytest_rc=$?" >> gpurun_out/pytest_gpu8.log; exit 3; }
timeout -k 10 300 python scripts/microbench.py --reps 20 > gpurun_out/micro8.log 2>&1 || exit 4
KCNN_FWD_VARIANT=1 timeout -k 10 100 python scripts/microbench.py --reps 20 --only fwd > gpurun_out/micro8_fwd1.log 2>&1 || exit 5
echo done
