set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest12.log 2>&1 || { echo "pytest_rc=$?" >> gpurun_out/pytest12.log; exit 3; }
timeout -k 10 100 python scripts/microbench.py --reps 20 --only pool_fwd,pool_bwd > gpurun_out/micro12.log 2>&1 || exit 5
echo done
