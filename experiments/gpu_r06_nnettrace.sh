# r06: one nnet.config step's kernel sequence (kernel trace, 3 timed steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r06nt; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --config nnet --steps 3 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1
