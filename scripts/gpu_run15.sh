set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/micro15.log
for d in 0 4096 8192 324 4420 8516; do
  echo "dbg=$d" >> gpurun_out/micro15.log
  KCNN_BWD_DEBUG=$d timeout -k 10 100 python scripts/microbench.py --reps 30 --only bwd_fused >> gpurun_out/micro15.log 2>&1 || exit 5
done
echo done
