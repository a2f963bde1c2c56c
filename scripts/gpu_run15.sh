set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/micro15.log
for d in 192 196 452 68 324; do
  echo "dbg=$d" >> gpurun_out/micro15.log
  KCNN_BWD_DEBUG=$d timeout -k 10 100 python scripts/microbench.py --reps 20 --only bwd_fused,bwd_fused_nodx,dgrad >> gpurun_out/micro15.log 2>&1 || exit 5
done
echo done
