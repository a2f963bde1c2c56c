# r05: nnet.config kernel trace with the fixup kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r05np}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --config nnet --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || exit 6
python scripts/kstats.py "$(find $O/prof -name "*kernel_stats.csv" | head -1)" 45 13
