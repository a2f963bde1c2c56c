set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in 0 4; do
KCNN_BWD_DEBUG=$d timeout -k 10 100 python scripts/microbench.py --reps 20 --only bwd_fused,bwd_fused_nodx > gpurun_out/micro11_$d.log 2>&1 || exit 5
done
echo done
