set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "conv or Conv or golden or dp or fd" > gpurun_out/pytest14.log 2>&1 || { echo "pytest_rc=$?" >> gpurun_out/pytest14.log; exit 3; }
timeout -k 10 200 python scripts/microbench.py --reps 20 --only bwd_fused,bwd_fused_nodx,dgrad > gpurun_out/micro14.log 2>&1 || exit 5
KCNN_BWD_DEBUG=32 timeout -k 10 200 python scripts/microbench.py --reps 20 --only bwd_fused >> gpurun_out/micro14.log 2>&1 || exit 6
KCNN_BWD_DEBUG=16 timeout -k 10 200 python scripts/microbench.py --reps 1 --only bwd_fused > gpurun_out/tm14.log 2>&1 || exit 7
echo done
