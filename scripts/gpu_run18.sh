set -o pipefail
O=gpurun_out/r18
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest_rc=$?" >> $O/pytest.log; exit 3; }
timeout -k 10 200 python scripts/microbench.py --reps 30 --only fwd,bwd_fused,bwd_fused_nodx,dgrad > $O/micro.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_default.log 2>&1 || exit 5
echo done
