# Round evidence on one MI355X: full GPU tests, smoke, bench lines (c2 with
# the CPU baseline, c5, nnet), rocprofv3 kernel stats of each, and the PMC
# HBM-traffic passes (FETCH_SIZE / WRITE_SIZE, one counter per pass) of c2.
#   scripts/gpu_profiles.sh <outdir>     (PART=1: tests, smoke and bench lines
#   only; PART=2: the rocprofv3 passes only, into the same <outdir>)
set -o pipefail
O=${1:-gpurun_out/profiles}
PART=${PART:-0}
if [ "$PART" != 2 ]; then rm -rf $O; fi
mkdir -p $O
export TMPDIR=/tmp
if [ "$PART" != 2 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest_rc=$?" >> $O/pytest_gpu.log; tail -30 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 4
timeout -k 10 600 python bench.py --json-out $O/bench.json > $O/bench.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --no-cpu-baseline --no-fusion --json-out $O/bench_nofusion.json > $O/bench_nofusion.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --no-cpu-baseline --store-conv-out --json-out $O/bench_store.json > $O/bench_store.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --config c5 --json-out $O/bench_c5.json > $O/bench_c5.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --config nnet --json-out $O/bench_nnet.json > $O/bench_nnet.log 2>&1 || exit 5
# c3 (65536 frames on one GPU) and one rank's c4 shard (16384 frames)
timeout -k 10 300 python bench.py --no-cpu-baseline --frames-per-gpu 65536 --json-out $O/bench_c3.json > $O/bench_c3.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --no-cpu-baseline --frames-per-gpu 16384 --json-out $O/bench_c4shard.json > $O/bench_c4shard.log 2>&1 || exit 5
# the same c4 shard as a data-parallel rank at world size 1 (RCCL; the DP
# step's own cost beside the single-GPU line)
HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29513 bench.py --gpus 1 --no-cpu-baseline --frames-per-gpu 16384 --json-out $O/bench_c4shard_dp1.json > $O/bench_c4shard_dp1.log 2>&1 || exit 5
fi
if [ "$PART" = 1 ]; then echo done; exit 0; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c2.prof.log 2>&1 || exit 6
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/c2/pmc_$c -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/c2.pmc_$c.log 2>&1 || exit 7
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2nf/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fusion > $O/c2nf.prof.log 2>&1 || exit 6
for cfg in c5 nnet; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$cfg/prof -o run -- python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/$cfg.prof.log 2>&1 || exit 6
done
echo done
