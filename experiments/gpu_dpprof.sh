# Kernel-level profile of the c2 step on the single-GPU path (python
# bench.py) and on the data-parallel path at world size 1 (torchrun, RCCL)
set -o pipefail
O=${1:-gpurun_out/dpprof}; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/single -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/single.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dp1 -o run -- python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline > $O/dp1.log 2>&1 || exit 7
# 23 steps per run: 3 warm-up + 2 x 10 timed
for r in single dp1; do
  f=$(find $O/$r -name "*kernel_stats.csv" | head -1)
  python scripts/kstats.py $f 23 30 > $O/$r.txt 2>&1; echo "== $r"; cat $O/$r.txt
done
