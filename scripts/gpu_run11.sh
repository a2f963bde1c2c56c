set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
KCNN_BWD_DEBUG=16 timeout -k 10 100 python scripts/microbench.py --reps 2 --only bwd_fused > gpurun_out/micro11.log 2>&1 || exit 5
echo done
