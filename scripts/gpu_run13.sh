set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "pool or Pool" > gpurun_out/pytest13.log 2>&1 || { echo "pytest_rc=$?" >> gpurun_out/pytest13.log; exit 3; }
timeout -k 10 100 python scripts/microbench.py --reps 20 --only pool_fwd,pool_bwd > gpurun_out/micro13.log 2>&1 || exit 5
KCNN_POOL_DIRECT=0 timeout -k 10 100 python scripts/microbench.py --reps 20 --only pool_fwd >> gpurun_out/micro13.log 2>&1 || exit 6
echo done
